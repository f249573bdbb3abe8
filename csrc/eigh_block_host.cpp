// Host driver of the native block-Jacobi eigensolver (csrc/eigh_block.hip):
// warm start, padding, the sweep loop with its once-per-sweep convergence
// read-back, and the final ascending sort (reference semantics,
// kfac/layers/eigen.py:294-347: eigenvalues ascending, eigenvectors in
// columns).
//
//   B0 = Q0^T A Q0  (Q0 = previous eigenbasis; hipBLASLt GEMMs) or A (cold)
//   sweeps of bj_round until no 64x64 pair block is above threshold
//   evals = sort(diag B), evecs = V[:, order]
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <hip/hip_runtime.h>

#include <vector>

namespace kfac {
int bj_block();
void bj_round(float* B, float* V, float* J, int* skip, int* active, const float* thr2,
              int64_t N, int batch, int round, int inner_sweeps, float noise,
              hipStream_t s);
void bj_sweep_end(int* active, int batch, hipStream_t s);
}  // namespace kfac

// A: [b, n, n] fp32 symmetric.  Q0: optional [b, n, n] orthogonal warm start
// (eigenvectors in columns).  Returns (evals [b, n] ascending, evecs [b, n, n]
// in columns, sweeps [b] int32: sweeps run until convergence, -1 = not
// converged within max_sweeps, active [b, max_sweeps]: non-skipped pairs per
// sweep).
std::vector<at::Tensor> block_jacobi_eigh(at::Tensor A, c10::optional<at::Tensor> Q0,
                                          int64_t max_sweeps, double tol,
                                          int64_t inner_sweeps, double noise, bool refine) {
  TORCH_CHECK(A.is_cuda() && A.scalar_type() == at::kFloat && A.dim() == 3 &&
                  A.size(1) == A.size(2),
              "block_jacobi_eigh: A must be a [b, n, n] fp32 GPU tensor");
  const int64_t b = A.size(0), n = A.size(1);
  c10::hip::HIPGuardMasqueradingAsCUDA g(A.device());
  hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const int64_t PBK = 2 * kfac::bj_block();
  const int64_t N = (n + PBK - 1) / PBK * PBK;
  const int k = (int)(N / kfac::bj_block());
  const int np = k / 2;
  auto opts = A.options();
  auto Bp = at::zeros({b, N, N}, opts);
  auto Vp = at::zeros({b, N, N}, opts);
  auto Bn = Bp.narrow(1, 0, n).narrow(2, 0, n);
  auto Vn = Vp.narrow(1, 0, n).narrow(2, 0, n);
  if (Q0.has_value() && Q0->defined()) {
    TORCH_CHECK(Q0->sizes() == A.sizes() && Q0->scalar_type() == at::kFloat,
                "block_jacobi_eigh: Q0 must match A");
    auto T = at::matmul(A, *Q0);
    auto Bw = at::matmul(Q0->transpose(1, 2), T);
    Bn.copy_(Bw);
    Bn.add_(Bw.transpose(1, 2)).mul_(0.5);
    Vn.copy_(*Q0);
  } else {
    Bn.copy_(A);
    Vn.diagonal(0, 1, 2).fill_(1.f);
  }
  if (N > n) Vp.diagonal(0, 1, 2).narrow(1, n, N - n).fill_(1.f);
  // per-pair threshold: tol^2 ||B||_F^2 / #pairs
  const double npairs = (double)k * (k - 1) / 2.0;
  auto thr2 = (Bp * Bp).sum({1, 2}).mul_(tol * tol / npairs).contiguous();
  auto J = at::empty({b, np, PBK, PBK}, opts);
  auto iopts = opts.dtype(at::kInt);
  auto skip = at::zeros({b, np}, iopts);
  auto active = at::zeros({b}, iopts);
  auto host = at::empty({b}, at::TensorOptions().dtype(at::kInt).pinned_memory(true));
  std::vector<int> sweeps(b, -1);
  std::vector<int> hist(b * max_sweeps, 0);  // active pairs per sweep
  int done = 0;
  for (int64_t sw = 0; sw < max_sweeps && done < b; ++sw) {
    for (int r = 0; r < k - 1; ++r) {
      kfac::bj_round(Bp.data_ptr<float>(), Vp.data_ptr<float>(), J.data_ptr<float>(),
                     skip.data_ptr<int>(), active.data_ptr<int>(), thr2.data_ptr<float>(), N,
                     (int)b, r, (int)inner_sweeps, (float)noise, s);
    }
    C10_HIP_CHECK(hipMemcpyAsync(host.data_ptr<int>(), active.data_ptr<int>(), b * sizeof(int),
                                 hipMemcpyDeviceToHost, s));
    kfac::bj_sweep_end(active.data_ptr<int>(), (int)b, s);
    C10_HIP_CHECK(hipStreamSynchronize(s));
    const int* h = host.data_ptr<int>();
    for (int64_t i = 0; i < b; ++i) hist[i * max_sweeps + sw] = h[i] < 0 ? 0 : h[i];
    for (int64_t i = 0; i < b; ++i) {
      if (h[i] <= 0 && sweeps[i] < 0) {
        sweeps[i] = (int)sw + 1;
        ++done;
      }
    }
  }
  at::Tensor evals, V = Vn;
  if (refine) {
    // one Newton-Schulz step restores orthonormality lost to rounding over
    // the sweeps, V <- V (3 I - V^T V) / 2, and the eigenvalues are the
    // Rayleigh quotients v_i^T A v_i of the refined vectors (the diagonal of
    // B has drifted by the same rounding)
    auto G = at::matmul(Vn.transpose(1, 2), Vn);
    G.mul_(-0.5).diagonal(0, 1, 2).add_(1.5);
    V = at::matmul(Vn, G);
    evals = (at::matmul(A, V) * V).sum(1);
  } else {
    evals = Bp.diagonal(0, 1, 2).narrow(1, 0, n);
  }
  auto sorted = evals.sort(/*dim=*/1, /*descending=*/false);
  auto order = std::get<1>(sorted);
  auto evecs = V.gather(2, order.unsqueeze(1).expand({b, n, n})).contiguous();
  auto sw_t = at::from_blob(sweeps.data(), {b}, at::TensorOptions().dtype(at::kInt)).clone();
  auto hist_t = at::from_blob(hist.data(), {b, max_sweeps}, at::TensorOptions().dtype(at::kInt)).clone();
  return {std::get<0>(sorted).contiguous(), evecs, sw_t, hist_t};
}
