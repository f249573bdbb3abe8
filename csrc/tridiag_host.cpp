// Host driver of the batched tridiagonal divide and conquer (csrc/tridiag.hip;
// float64 CPU reference: distributed_kfac_pytorch_amd/ops/tridiag.py).
//
//   pad n -> n_pad = leaf * 2^levels (leaf <= 64, padding < 3 %; padded
//   diagonal above every eigenvalue, decoupled) -> leaves (dense leaf x leaf
//   blocks, LDS Jacobi kernel) -> per level: dc_merge_front (sort, deflation,
//   secular roots, z^), one batched sort of the merged values (output order),
//   dc_merge_back (W), Q = diag(Q1, Q2) W as ONE batched fp32 GEMM -> drop the
//   padding.  No host synchronisation.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <hip/hip_runtime.h>

#include <cmath>
#include <vector>

namespace kfac {
int dc_leaf_max();
int dc_max_m();
void dc_leaves(const float* d_pad, const float* e_pad, int batch, int n_pad, int leaf,
               float* out, hipStream_t s);
void dc_merge_front(const double* Dprev, const float* Qprev, const float* e_pad, int n_pad,
                    int h, int S, int G, double* sd, double* sz, int* perm, double* scal,
                    int* isnd, int* ndidx, int* rot_idx, double* rot_cs, int* cnt,
                    double* tau, double* zh, double* vals, hipStream_t s);
void dc_merge_back(int h, int G, const double* sd, const int* perm, const int* isnd,
                   const int* ndidx, const int* cnt, const double* tau, const double* zh,
                   const int64_t* outpos, const int* rot_idx, const double* rot_cs, float* W,
                   hipStream_t s);
void jacobi_eigh_batched(const float* A, int64_t n, int64_t batch, int64_t strideA,
                         float* evals, float* evecs, int64_t strideV, int max_sweeps, float tol,
                         hipStream_t s);
void gemm_f32_batched(int ta, int tb, int M, int N, int K, float alpha, const float* A,
                      int64_t lda, int64_t sA, const float* B, int64_t ldb, int64_t sB,
                      float beta, float* C, int64_t ldc, int64_t sC, int batch,
                      hipStream_t s, float* ws, int64_t ws_floats);
int64_t gemm_f32_ws_floats(int M, int N, int K, int batch);
}  // namespace kfac

namespace {
// native fp32 MFMA GEMM (csrc/gemm_f32.hip) with its split-K workspace
void gemm_native(int ta, int tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
                 int64_t lda, int64_t sA, const float* B, int64_t ldb, int64_t sB, float beta,
                 float* C, int64_t ldc, int64_t sC, int64_t batch, hipStream_t s,
                 const at::TensorOptions& opt) {
  const int64_t wsf = kfac::gemm_f32_ws_floats((int)M, (int)N, (int)K, (int)batch);
  at::Tensor ws;
  if (wsf > 0) ws = at::empty({wsf}, opt.dtype(at::kFloat));
  kfac::gemm_f32_batched(ta, tb, (int)M, (int)N, (int)K, alpha, A, lda, sA, B, ldb, sB, beta, C,
                         ldc, sC, (int)batch, s, wsf > 0 ? ws.data_ptr<float>() : nullptr, wsf);
}
}  // namespace


namespace {

struct Plan {
  int64_t leaf, levels, n_pad;
};

Plan dc_plan(int64_t n) {
  const int64_t L = kfac::dc_leaf_max();
  if (n <= L) return {n, 0, n};
  int64_t k = (int64_t)std::ceil(std::log2((double)n / (double)L));
  while ((L << k) < n) ++k;
  const int64_t leaf = (n + (int64_t(1) << k) - 1) >> k;
  return {leaf, k, leaf << k};
}

}  // namespace

// d [b, n], e [b, n-1] fp32 on the GPU (diagonal / off-diagonal of b
// symmetric tridiagonal matrices).  Returns (w [b, n] ascending, Z [b, n, n]
// eigenvectors in columns), fp32.
std::vector<at::Tensor> tridiag_eigh_dc(const at::Tensor& d_in, const at::Tensor& e_in) {
  TORCH_CHECK(d_in.is_cuda() && d_in.dim() == 2, "tridiag_eigh_dc: d must be [b, n] on the GPU");
  const int64_t b = d_in.size(0), n = d_in.size(1);
  TORCH_CHECK(e_in.dim() == 2 && e_in.size(0) == b && e_in.size(1) == std::max<int64_t>(n - 1, 0),
              "tridiag_eigh_dc: e must be [b, n-1]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(d_in.device());
  hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  auto fopt = d_in.options().dtype(at::kFloat);
  const at::Tensor d = d_in.to(at::kFloat).contiguous();
  const at::Tensor e = e_in.to(at::kFloat).contiguous();
  const Plan pl = dc_plan(n);
  TORCH_CHECK(pl.n_pad <= kfac::dc_max_m(), "tridiag_eigh_dc supports n <= ", kfac::dc_max_m());
  if (b == 0 || n == 0) return {at::empty({b, n}, fopt), at::empty({b, n, n}, fopt)};
  // padding: decoupled diagonal entries above the Gershgorin bound
  at::Tensor dp = d, ep = e;
  if (pl.n_pad > n) {
    auto rad = at::zeros_like(d);
    if (n > 1) {
      auto ae = e.abs();
      rad.narrow(1, 0, n - 1).add_(ae);
      rad.narrow(1, 1, n - 1).add_(ae);
    }
    auto g = (d + rad).amax(1, true);
    auto pv = g + g.abs().clamp_min(1.0);
    dp = at::cat({d, pv.expand({b, pl.n_pad - n})}, 1).contiguous();
    ep = at::cat({e, at::zeros({b, pl.n_pad - 1 - (n - 1)}, fopt)}, 1).contiguous();
  }
  const int64_t L = pl.leaf, np = pl.n_pad;
  const int64_t nl = np / L;
  auto blocks = at::empty({b * nl, L, L}, fopt);
  if (np > 1) {
    kfac::dc_leaves(dp.data_ptr<float>(), ep.data_ptr<float>(), (int)b, (int)np, (int)L,
                    blocks.data_ptr<float>(), s);
  } else {
    blocks.copy_(dp.view({b, 1, 1}));
  }
  auto wl = at::empty({b * nl, L}, fopt);
  auto Q = at::empty({b * nl, L, L}, fopt);
  kfac::jacobi_eigh_batched(blocks.data_ptr<float>(), L, b * nl, L * L, wl.data_ptr<float>(),
                            Q.data_ptr<float>(), L * L, 30, 1e-7f, s);
  at::Tensor D = wl.to(at::kDouble);  // [G_child, h] ascending
  auto iopt = d_in.options().dtype(at::kInt);
  auto dopt = d_in.options().dtype(at::kDouble);
  for (int64_t lv = 0; lv < pl.levels; ++lv) {
    const int64_t h = L << lv, m = 2 * h;
    const int64_t S = np / m, G = b * S;
    auto sd = at::empty({G, m}, dopt);
    auto sz = at::empty({G, m}, dopt);
    auto perm = at::empty({G, m}, iopt);
    auto scal = at::empty({G, 4}, dopt);
    auto isnd = at::empty({G, m}, iopt);
    auto ndidx = at::empty({G, m}, iopt);
    auto rot_idx = at::empty({G, m, 2}, iopt);
    auto rot_cs = at::empty({G, m, 2}, dopt);
    auto cnt = at::empty({G, 2}, iopt);
    auto tau = at::empty({G, m}, dopt);
    auto zh = at::empty({G, m}, dopt);
    auto vals = at::empty({G, m}, dopt);
    const at::Tensor Dc = D.view({G, m}).contiguous();
    kfac::dc_merge_front(Dc.data_ptr<double>(), Q.data_ptr<float>(), ep.data_ptr<float>(),
                         (int)np, (int)h, (int)S, (int)G, sd.data_ptr<double>(),
                         sz.data_ptr<double>(), perm.data_ptr<int>(), scal.data_ptr<double>(),
                         isnd.data_ptr<int>(), ndidx.data_ptr<int>(), rot_idx.data_ptr<int>(),
                         rot_cs.data_ptr<double>(), cnt.data_ptr<int>(), tau.data_ptr<double>(),
                         zh.data_ptr<double>(), vals.data_ptr<double>(), s);
    auto sorted = at::sort(vals, /*stable=*/true, /*dim=*/1, /*descending=*/false);
    const at::Tensor& svals = std::get<0>(sorted);
    const at::Tensor& order = std::get<1>(sorted);
    auto outpos = at::empty_like(order);
    outpos.scatter_(1, order, at::arange(m, order.options()).expand({G, m}));
    auto W = at::zeros({G, m, m}, fopt);
    kfac::dc_merge_back((int)h, (int)G, sd.data_ptr<double>(), perm.data_ptr<int>(),
                        isnd.data_ptr<int>(), ndidx.data_ptr<int>(), cnt.data_ptr<int>(),
                        tau.data_ptr<double>(), zh.data_ptr<double>(),
                        outpos.data_ptr<int64_t>(), rot_idx.data_ptr<int>(),
                        rot_cs.data_ptr<double>(), W.data_ptr<float>(), s);
    // Q_parent = diag(Q1, Q2) W: the two row halves of every subproblem are
    // the children's blocks times W's row halves
    auto Qn = at::empty({G, m, m}, fopt);
    gemm_native(0, 0, (int)h, (int)m, (int)h, 1.f, Q.data_ptr<float>(), h, h * h,
                           W.data_ptr<float>(), m, h * m, 0.f, Qn.data_ptr<float>(), m, h * m,
                           (int)(2 * G), s, fopt);
    Q = Qn;
    D = svals;
  }
  auto w = D.view({b, np}).narrow(1, 0, n).to(at::kFloat).contiguous();
  auto Z = Q.view({b, np, np}).narrow(1, 0, n).narrow(2, 0, n).contiguous();
  return {w, Z};
}

// (leaf, levels, n_pad) of the padded tree (tests / tools)
std::vector<int64_t> tridiag_dc_plan(int64_t n) {
  const Plan p = dc_plan(n);
  return {p.leaf, p.levels, p.n_pad};
}
