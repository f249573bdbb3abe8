// Host driver of the two-stage batched symmetric eigensolver (K-HIP-3):
//
//   dense -> band (csrc/sy2sb.hip panel QR + batched GEMM two-sided updates)
//   band -> tridiagonal (csrc/sb2st.hip bulge chasing, one workgroup per matrix)
//   tridiagonal eigenpairs (csrc/tridiag.hip divide and conquer)
//   X = Q2 Z (csrc/bt2.hip, one launch per step of disjoint rank-16 blocks)
//   X = Q1 X (blocked UT back-transform, 512 reflectors per block: native
//   fp32 MFMA GEMMs and triangular inverse, csrc/gemm_f32.hip)
//
// for a batch of same-size fp32 symmetric matrices, all on the current
// stream, no host synchronisation.  Reference: torch.linalg.eigh in
// kfac/layers/eigen.py:294-347.  float64 oracle of every stage:
// distributed_kfac_pytorch_amd/ops/twostage.py.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <limits>
#include <vector>

namespace kfac {
int twostage_band();
int twostage_max_n();
void sb_panel_qr(float* A, int64_t sA, int ld, int n, int p, int batch, float* Vw, float* Uw,
                 int64_t sVU, float* tau1, int64_t sTau, float* Tw, hipStream_t stream);
void sb_update_front(float* A, int64_t sA, int ld, int n, int p, int batch, const float* Vw,
                     const float* Uw, int64_t sVU, const float* Tw, float* Ypart, float* Spart,
                     float* Ms, float* Ww, hipStream_t stream);
bool sb_update_back(float* A, int64_t sA, int ld, int n, int p, int batch, const float* Vw,
                    int64_t sVU, const float* Ww, hipStream_t stream);
void sb_extract(const float* A, int64_t sA, int ld, int n, int batch, float* AB, int64_t sAB,
                int ncols, hipStream_t stream);
int sb2st_kmax(int n);
void sb2st(float* AB, int64_t sAB, int n, int batch, float* V2, float* tau2, int64_t sV2,
           int kmax, float* d, float* e, int* err, hipStream_t stream);
int bt2_groups(int n);
void bt2_prep(const float* V2, const float* tau2, int64_t sV2, int n, int kmax, int batch,
              float* T, hipStream_t stream);
void bt2_apply(const float* V2, int64_t sV2, const float* T, int n, int kmax, int batch,
               float* X, int64_t sX, int ldx, hipStream_t stream);
void gemm_f32_batched(int ta, int tb, int M, int N, int K, float alpha, const float* A,
                      int64_t lda, int64_t sA, const float* B, int64_t ldb, int64_t sB,
                      float beta, float* C, int64_t ldc, int64_t sC, int batch,
                      hipStream_t s, float* ws, int64_t ws_floats);
int64_t gemm_f32_ws_floats(int M, int N, int K, int batch);
void trinv_upper_batched(float* T, int64_t ld, int64_t sT, int n, int batch, float* work,
                         hipStream_t s);
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


std::vector<at::Tensor> tridiag_eigh_dc(const at::Tensor& d, const at::Tensor& e);

namespace {

hipStream_t cur() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

// stage-1 reflector k (k = 0 .. nref-1) lives in COLUMN k of A below the
// band: v[k+16] = 1 implicit, v[k+17 ..] stored; X <- Q1 X with Q1 = H_0 H_1 ... H_{nref-1},
// nb reflectors per UT block (T^-1 = striu(V^T V) + diag(1/tau)), last block
// first.
void apply_q1(const at::Tensor& A, const at::Tensor& tau1, int64_t n, int64_t nref,
              at::Tensor& X, int64_t nb) {
  const int64_t off = kfac::twostage_band();
  auto fopt = X.options();
  const int64_t b = X.size(0);
  for (int64_t p0 = ((nref - 1) / nb) * nb; p0 >= 0; p0 -= nb) {
    const int64_t p1 = std::min(p0 + nb, nref);
    const int64_t bs = p1 - p0;
    const int64_t rows = n - p0 - off;
    if (rows <= 0) continue;
    // reflector p0+kk in column p0+kk below the band: vt[kk][j] = A[p0+off+j][p0+kk]
    auto W = A.narrow(2, p0, bs).narrow(1, p0 + off, rows).transpose(1, 2);
    auto vt = at::triu(W, 1);
    auto t = tau1.narrow(1, p0, bs);
    auto live = t.ne(0).to(at::kFloat);
    auto eye_bs = at::eye(bs, rows, fopt).unsqueeze(0);
    vt = (vt + eye_bs) * live.unsqueeze(2);
    vt = vt.contiguous();
    auto g = at::empty({b, bs, bs}, fopt);  // V V^T (native fp32 MFMA)
    gemm_native(0, 1, (int)bs, (int)bs, (int)rows, 1.f, vt.data_ptr<float>(), rows,
                           bs * rows, vt.data_ptr<float>(), rows, bs * rows, 0.f,
                           g.data_ptr<float>(), bs, bs * bs, (int)b, cur(), fopt);
    auto dinv = at::where(t.eq(0), at::ones_like(t), at::reciprocal(at::where(t.eq(0),
                                                                                at::ones_like(t), t)));
    auto u = at::triu(g, 1) + at::diag_embed(dinv);
    // tm = u^-1 (u upper triangular, row-major) by rocBLAS trsm on the
    // column-major view (u^T, lower): the result read row-major is u^-1
    // tm = u^-1 (u upper triangular): native blocked triangular inverse
    auto tm = u.contiguous();
    {
      auto work = at::empty({std::max<int64_t>(b * bs * bs / 2 + bs, 1)}, fopt);
      kfac::trinv_upper_batched(tm.data_ptr<float>(), bs, bs * bs, (int)bs, (int)b,
                                work.data_ptr<float>(), cur());
    }
    // rows p0+off.. of X in place (leading dimension n), native fp32 MFMA:
    // W1 = vt Xs ([bs, rows] x [rows, n]), W2 = tm W1, Xs -= vt^T W2
    vt = vt.contiguous();
    float* xs = X.data_ptr<float>() + (p0 + off) * n;
    auto w1 = at::empty({b, bs, n}, fopt);
    auto w2 = at::empty({b, bs, n}, fopt);
    gemm_native(0, 0, (int)bs, (int)n, (int)rows, 1.f, vt.data_ptr<float>(), rows,
                           bs * rows, xs, n, n * n, 0.f, w1.data_ptr<float>(), n, bs * n,
                           (int)b, cur(), fopt);
    gemm_native(0, 0, (int)bs, (int)n, (int)bs, 1.f, tm.data_ptr<float>(), bs,
                           bs * bs, w1.data_ptr<float>(), n, bs * n, 0.f,
                           w2.data_ptr<float>(), n, bs * n, (int)b, cur(), fopt);
    gemm_native(1, 0, (int)rows, (int)n, (int)bs, -1.f, vt.data_ptr<float>(), rows,
                           bs * rows, w2.data_ptr<float>(), n, bs * n, 1.f, xs, n, n * n,
                           (int)b, cur(), fopt);
  }
}

}  // namespace

int64_t eigh_twostage_max_n() { return kfac::twostage_max_n(); }

// A [b, n, n] fp32 symmetric on the GPU -> (w [b, n] ascending, X [b, n, n]
// eigenvectors in columns, err [batch] int32: nonzero if the bulge-chasing
// pipeline timed out -- then w is NaN).  `times` (optional, host fp32 [5]):
// per-stage milliseconds (synchronises; diagnostics only).
std::vector<at::Tensor> eigh_twostage(const at::Tensor& A_in, bool timed) {
  TORCH_CHECK(A_in.is_cuda() && A_in.dim() == 3 && A_in.size(1) == A_in.size(2),
              "eigh_twostage: A must be [b, n, n] on the GPU");
  const int64_t b = A_in.size(0), n = A_in.size(1);
  const int64_t B = kfac::twostage_band();
  TORCH_CHECK(n >= 3 && n <= kfac::twostage_max_n(), "eigh_twostage: 3 <= n <= ",
              kfac::twostage_max_n());
  c10::hip::HIPGuardMasqueradingAsCUDA guard(A_in.device());
  hipStream_t s = cur();
  auto fopt = A_in.options().dtype(at::kFloat);
  std::vector<hipEvent_t> ev;
  auto mark = [&]() {
    if (!timed) return;
    hipEvent_t e;
    hipEventCreate(&e);
    hipEventRecord(e, s);
    ev.push_back(e);
  };
  mark();
  const int64_t ld = (n + 3) / 4 * 4;
  auto A = at::zeros({b, n, ld}, fopt);
  A.narrow(2, 0, n).copy_(A_in);
  // double-buffered panel operands (panel parity): the next panel's QR writes
  // one set while this panel's back update (side stream) reads the other
  auto Vw = at::empty({2, b, n, B}, fopt);
  auto Uw = at::empty({2, b, n, B}, fopt);
  auto Ww = at::empty({2, b, n, B}, fopt);
  auto Tw = at::empty({2, b, B, B}, fopt);
  auto tau1 = at::zeros({b, n}, fopt);
  int64_t nref = 0;
  const int64_t nblk = (n + 63) / 64;
  auto Ypart = at::empty({8, b, n, B}, fopt);
  auto Spart = at::empty({b, nblk * 8, B * B}, fopt);
  auto Ms = at::empty({b, B, B}, fopt);
  // ---- stage 1: panel p's QR and the front of its update on s; the rest of
  // its trailing update on the side stream, overlapping panel p+1's QR
  hipStream_t side = c10::hip::getStreamFromPool(false, A_in.device().index()).stream();
  hipEvent_t ev_front, ev_back;
  C10_HIP_CHECK(hipEventCreateWithFlags(&ev_front, hipEventDisableTiming));
  C10_HIP_CHECK(hipEventCreateWithFlags(&ev_back, hipEventDisableTiming));
  bool back_pending = false;
  for (int64_t p = 0; n - p - B >= 2; p += B) {
    const int par = (int)((p / B) & 1);
    float* vw = Vw[par].data_ptr<float>();
    float* uw = Uw[par].data_ptr<float>();
    float* ww = Ww[par].data_ptr<float>();
    float* tw = Tw[par].data_ptr<float>();
    kfac::sb_panel_qr(A.data_ptr<float>(), n * ld, (int)ld, (int)n, (int)p, (int)b, vw, uw,
                      n * B, tau1.data_ptr<float>(), n, tw, s);
    nref = p + B;
    if (back_pending) C10_HIP_CHECK(hipStreamWaitEvent(s, ev_back, 0));
    kfac::sb_update_front(A.data_ptr<float>(), n * ld, (int)ld, (int)n, (int)p, (int)b, vw, uw,
                          n * B, tw, Ypart.data_ptr<float>(), Spart.data_ptr<float>(),
                          Ms.data_ptr<float>(), ww, s);
    C10_HIP_CHECK(hipEventRecord(ev_front, s));
    C10_HIP_CHECK(hipStreamWaitEvent(side, ev_front, 0));
    back_pending = kfac::sb_update_back(A.data_ptr<float>(), n * ld, (int)ld, (int)n, (int)p,
                                        (int)b, vw, n * B, ww, side);
    if (back_pending) C10_HIP_CHECK(hipEventRecord(ev_back, side));
  }
  if (back_pending) C10_HIP_CHECK(hipStreamWaitEvent(s, ev_back, 0));
  C10_HIP_CHECK(hipEventDestroy(ev_front));
  C10_HIP_CHECK(hipEventDestroy(ev_back));
  mark();
  // ---- stage 2
  const int64_t ncols = n + 4 * B;
  auto AB = at::empty({b, ncols, 2 * B}, fopt);
  kfac::sb_extract(A.data_ptr<float>(), n * ld, (int)ld, (int)n, (int)b, AB.data_ptr<float>(),
                   ncols * 2 * B, (int)ncols, s);
  const int kmax = kfac::sb2st_kmax((int)n);
  const int64_t nslot = (n - 2) * kmax;
  auto V2 = at::zeros({b, nslot, B}, fopt);
  auto tau2 = at::zeros({b, nslot}, fopt);
  auto d = at::empty({b, n}, fopt);
  auto e = at::empty({b, n - 1}, fopt);
  // one timeout flag per matrix: a timed-out pipeline poisons only its own
  // eigenvalues (and so only its own repair in ops.linalg)
  auto err = at::zeros({b}, A_in.options().dtype(at::kInt));
  kfac::sb2st(AB.data_ptr<float>(), ncols * 2 * B, (int)n, (int)b, V2.data_ptr<float>(),
              tau2.data_ptr<float>(), nslot, kmax, d.data_ptr<float>(), e.data_ptr<float>(),
              err.data_ptr<int>(), s);
  // a timed-out pipeline must never be installed: poison its eigenvalues
  d = at::where(err.ne(0).unsqueeze(1), at::full({}, std::numeric_limits<float>::quiet_NaN(), fopt),
                d);
  mark();
  // ---- tridiagonal eigenpairs
  auto wz = tridiag_eigh_dc(d, e);
  at::Tensor w = wz[0];
  at::Tensor X = wz[1].contiguous();
  mark();
  // ---- back-transforms
  const int G = kfac::bt2_groups((int)n);
  auto T2 = at::empty({b, (int64_t)G * kmax, B, B}, fopt);
  kfac::bt2_prep(V2.data_ptr<float>(), tau2.data_ptr<float>(), nslot, (int)n, kmax, (int)b,
                 T2.data_ptr<float>(), s);
  kfac::bt2_apply(V2.data_ptr<float>(), nslot, T2.data_ptr<float>(), (int)n, kmax, (int)b,
                  X.data_ptr<float>(), n * n, (int)n, s);
  mark();
  if (nref > 0) apply_q1(A, tau1, n, nref, X, 512);
  mark();
  at::Tensor times = at::zeros({std::max<int64_t>((int64_t)ev.size() - 1, 0)},
                               at::TensorOptions().dtype(at::kFloat));
  if (timed) {
    hipEventSynchronize(ev.back());
    for (size_t i = 0; i + 1 < ev.size(); ++i) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, ev[i], ev[i + 1]);
      times[i].fill_(ms);
    }
    for (auto& x : ev) hipEventDestroy(x);
  }
  return {w, X, err, times};
}
