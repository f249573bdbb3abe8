// Large-factor eigensolver tier: direct rocSOLVER calls (syevd / syevj /
// syevdj, strided-batched) on a caller-chosen HIP stream.
//
// Compared with torch.linalg.eigh this (a) never synchronises the host (the
// per-matrix `info` stays on the device; torch checks it with a blocking
// copy after every call), so several size buckets can be in flight on
// different streams at once, and (b) lets K-FAC pick the algorithm per size:
// Jacobi (syevj) for batches of mid-size factors, divide & conquer (syevd)
// for the large ones.  Workspace comes from the torch caching allocator and
// is bound to a rocBLAS handle cached per stream, so steady-state calls do no
// hipMalloc.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include "descs.h"

#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

struct HandleState {
  rocblas_handle handle = nullptr;
  at::Tensor workspace;
};

// Intentionally leaked: destroying the map at static-destruction time would
// free device workspaces after the HIP runtime / torch allocator have been
// torn down (heap corruption at interpreter exit).
std::mutex g_mu;
std::unordered_map<hipStream_t, HandleState>& g_handles =
    *new std::unordered_map<hipStream_t, HandleState>();

#define ROCBLAS_OK(expr)                                                   \
  do {                                                                     \
    rocblas_status _s = (expr);                                            \
    TORCH_CHECK(_s == rocblas_status_success, "rocSOLVER/rocBLAS error ",  \
                (int)_s, " in ", #expr);                                   \
  } while (0)

HandleState& handle_for(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_handles.find(s);
  if (it != g_handles.end()) return it->second;
  HandleState st;
  ROCBLAS_OK(rocblas_create_handle(&st.handle));
  ROCBLAS_OK(rocblas_set_stream(st.handle, s));
  return g_handles.emplace(s, std::move(st)).first->second;
}

enum Algo : int64_t { kSyevd = 0, kSyevj = 1, kSyevdj = 2 };

rocblas_status call(rocblas_handle h, int64_t algo, int n, float* A,
                    int64_t strideA, float* W, int64_t strideW, float* E,
                    int* info,
                    float* residual, int* nsweeps, int max_sweeps, float tol,
                    int batch) {
  switch (algo) {
    case kSyevj:
      return rocsolver_ssyevj_strided_batched(
          h, rocblas_esort_ascending, rocblas_evect_original,
          rocblas_fill_upper, n, A, n, strideA, tol, residual, max_sweeps,
          nsweeps, W, strideW, info, batch);
    case kSyevdj:
      return rocsolver_ssyevdj_strided_batched(
          h, rocblas_evect_original, rocblas_fill_upper, n, A, n, strideA, W,
          strideW, info, batch);
    default:
      return rocsolver_ssyevd_strided_batched(
          h, rocblas_evect_original, rocblas_fill_upper, n, A, n, strideA, W,
          strideW, E, n, info, batch);
  }
}

}  // namespace

// A: [batch, n, n] fp32 contiguous symmetric; overwritten with eigenvectors.
// Returns (evals [batch, n] ascending, evecs [batch, n, n] with eigenvectors
// in columns -- a transposed view of the column-major rocSOLVER output).
std::vector<at::Tensor> rocsolver_eigh(at::Tensor A, int64_t algo,
                                       int64_t max_sweeps, double tol) {
  TORCH_CHECK(A.is_cuda() && A.scalar_type() == at::kFloat && A.dim() == 3 &&
              A.size(1) == A.size(2) && A.is_contiguous());
  const int64_t batch = A.size(0), n = A.size(1);
  c10::hip::HIPGuardMasqueradingAsCUDA g(A.device());
  hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  auto W = at::empty({batch, n}, A.options());
  auto ints = at::empty({2 * batch}, A.options().dtype(at::kInt));
  auto resid = at::empty({batch}, A.options());
  auto E = at::empty({batch, n}, A.options());
  if (batch == 0 || n == 0) return {W, A.transpose(1, 2)};
  HandleState& st = handle_for(s);
  // workspace size query, then bind a torch-allocated workspace
  size_t need = 0;
  ROCBLAS_OK(rocblas_start_device_memory_size_query(st.handle));
  call(st.handle, algo, (int)n, A.data_ptr<float>(), n * n, W.data_ptr<float>(),
       n, E.data_ptr<float>(), ints.data_ptr<int>(), resid.data_ptr<float>(),
       ints.data_ptr<int>() + batch, (int)max_sweeps, (float)tol, (int)batch);
  ROCBLAS_OK(rocblas_stop_device_memory_size_query(st.handle, &need));
  if (!st.workspace.defined() || (size_t)st.workspace.numel() < need) {
    st.workspace = at::empty({(int64_t)std::max<size_t>(need, 1)},
                             A.options().dtype(at::kByte));
    ROCBLAS_OK(rocblas_set_workspace(st.handle, st.workspace.data_ptr(),
                                     (size_t)st.workspace.numel()));
  }
  ROCBLAS_OK(call(st.handle, algo, (int)n, A.data_ptr<float>(), n * n,
                  W.data_ptr<float>(), n, E.data_ptr<float>(),
                  ints.data_ptr<int>(),
                  resid.data_ptr<float>(), ints.data_ptr<int>() + batch,
                  (int)max_sweeps, (float)tol, (int)batch));
  return {W, A.transpose(1, 2)};
}

// ---------------------------------------------------------------------------
// Large-n tier built on the native batched tridiagonalisation (sytrd.hip):
// sytrd_reduce() reduces every matrix of every bucket in ONE launch chain
// (in place: reflectors in the rows of A, d / e / tau out), then
// tridiag_eigvecs() finishes one bucket with rocSOLVER stedc (divide and
// conquer on T, eigenvectors of T) + ormtr (Z = Q Z_T), i.e. exactly the
// second half of syevd.  Buckets can be finished on different streams.
namespace kfac {
int sytrd_nb();
int sytrd_max_n();
int sytrd_p1();
int sytrd_maxch();
int sytrd_maxrowblk();
void sytrd_batched(const SytrdDesc* descs_dev, const int* ns, int batch,
                   hipStream_t stream);
void sytrd_batched_range(const SytrdDesc* descs_dev, const int* ns, int batch,
                         int k_begin, int k_end, hipStream_t stream, int waves);
}  // namespace kfac

int64_t sytrd_max_n() { return kfac::sytrd_max_n(); }
int64_t sytrd_panel() { return kfac::sytrd_nb(); }

// stacks: list of [cnt, n, n] fp32 contiguous symmetric (overwritten).
// Descriptor table + workspace for a reduction of `stacks`; returns
// [descs (device bytes), work, d0, e0, tau0, d1, ...].  Nothing launched.
static std::vector<at::Tensor> sytrd_setup(std::vector<at::Tensor>& stacks,
                                           std::vector<int>& ns) {
  TORCH_CHECK(!stacks.empty());
  const auto opts = stacks[0].options();
  const int NB = kfac::sytrd_nb(), P1 = kfac::sytrd_p1();
  std::vector<at::Tensor> outs;
  int64_t scratch = 0;
  for (auto& A : stacks) {
    TORCH_CHECK(A.is_cuda() && A.scalar_type() == at::kFloat && A.dim() == 3 &&
                A.size(1) == A.size(2) && A.is_contiguous());
    TORCH_CHECK(A.size(1) <= kfac::sytrd_max_n(), "sytrd supports n <= ",
                kfac::sytrd_max_n());
    const int64_t cnt = A.size(0), n = A.size(1);
    for (int64_t b = 0; b < cnt; ++b) ns.push_back((int)n);
    scratch += cnt * ((int64_t)NB * n + (int64_t)kfac::sytrd_maxch() * P1 +
                      kfac::sytrd_maxrowblk() + 4 + 2 * NB);
  }
  const int batch = (int)ns.size();
  if (batch == 0) return outs;
  auto work = at::empty({std::max<int64_t>(scratch, 1)}, opts);
  float* wp = work.data_ptr<float>();
  auto host = at::empty({(int64_t)(batch * sizeof(kfac::SytrdDesc))},
                        at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  auto* descs = reinterpret_cast<kfac::SytrdDesc*>(host.data_ptr());
  int idx = 0;
  for (auto& A : stacks) {
    const int64_t cnt = A.size(0), n = A.size(1);
    auto d = at::empty({cnt, n}, opts), e = at::zeros({cnt, n}, opts),
         tau = at::zeros({cnt, n}, opts);
    for (int64_t b = 0; b < cnt; ++b) {
      kfac::SytrdDesc& D = descs[idx++];
      D.A = A.data_ptr<float>() + b * n * n;
      D.d = d.data_ptr<float>() + b * n;
      D.e = e.data_ptr<float>() + b * n;
      D.tau = tau.data_ptr<float>() + b * n;
      D.Wt = wp;
      wp += (int64_t)NB * n;
      D.part1 = wp;
      wp += (int64_t)kfac::sytrd_maxch() * P1;
      D.part2 = wp;
      wp += kfac::sytrd_maxrowblk();
      D.sc = wp;
      wp += 4 + 2 * NB;
      D.P = nullptr;
      D.n = (int)n;
      D.pad = 0;
    }
    outs.push_back(d);
    outs.push_back(e);
    outs.push_back(tau);
  }
  auto dev = at::empty({host.numel()}, opts.dtype(at::kByte));
  dev.narrow(0, 0, host.numel()).copy_(host, /*non_blocking=*/true);
  outs.insert(outs.begin(), work);
  outs.insert(outs.begin(), dev);
  return outs;
}

std::vector<at::Tensor> sytrd_reduce(std::vector<at::Tensor> stacks) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(stacks.at(0).device());
  hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  std::vector<int> ns;
  auto all = sytrd_setup(stacks, ns);
  if (ns.empty()) return {};
  kfac::sytrd_batched(reinterpret_cast<const kfac::SytrdDesc*>(all[0].data_ptr()),
                      ns.data(), (int)ns.size(), s);
  return std::vector<at::Tensor>(all.begin() + 2, all.end());
}

// Segmented form: sytrd_begin() builds the state (kept alive by the caller
// in the returned tensors: [descs, work, d0, e0, tau0, ...]); each
// sytrd_advance(state, sizes, k0, k1) issues the panels covering columns
// [k0, k1) (k0 a multiple of the panel width) on the current stream.  After
// advancing past n, every matrix of size <= n is fully reduced.  `waves`
// sizes each symv launch (0: the whole chip, see sytrd_symv_blocks).
std::vector<at::Tensor> sytrd_begin(std::vector<at::Tensor> stacks) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(stacks.at(0).device());
  std::vector<int> ns;
  return sytrd_setup(stacks, ns);
}

void sytrd_advance(at::Tensor descs, std::vector<int64_t> sizes, int64_t k0, int64_t k1,
                   int64_t waves) {
  TORCH_CHECK(k0 % kfac::sytrd_nb() == 0, "segments start on panel boundaries");
  c10::hip::HIPGuardMasqueradingAsCUDA g(descs.device());
  hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  std::vector<int> ns(sizes.begin(), sizes.end());
  TORCH_CHECK((int64_t)ns.size() * (int64_t)sizeof(kfac::SytrdDesc) ==
              descs.numel());
  kfac::sytrd_batched_range(reinterpret_cast<const kfac::SytrdDesc*>(descs.data_ptr()),
                            ns.data(), (int)ns.size(), (int)k0, (int)k1, s, (int)waves);
}

// ---------------------------------------------------------------------------
// K-HIP-5 blocked tier (csrc/spdinv_chol.hip): blocked Cholesky + triangular
// inverse + W^T W on fp32 MFMA tiles, any n.  Returns (X [cnt, n, n] exactly
// symmetric, failed [cnt] int32: 1 where a Cholesky pivot was non-positive /
// non-finite -- the caller re-solves those with a pivoted LU so no NaN is
// ever installed).
namespace kfac {
int64_t spd_chol_pad(int64_t n);
void spd_inverse_chol(const float* F, float* X, float* M, float* W, float* Linv, int* fail,
                      int64_t n, int batch, float damping, hipStream_t s);
}  // namespace kfac

std::vector<at::Tensor> spd_inverse_blocked(at::Tensor F, double damping) {
  TORCH_CHECK(F.is_cuda() && F.scalar_type() == at::kFloat && F.dim() == 3 &&
              F.size(1) == F.size(2) && F.is_contiguous());
  const int64_t cnt = F.size(0), n = F.size(1);
  c10::hip::HIPGuardMasqueradingAsCUDA g(F.device());
  hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  auto X = at::empty_like(F);
  auto fail = at::zeros({cnt}, F.options().dtype(at::kInt));
  if (cnt == 0 || n == 0) return {X, fail};
  const int64_t N = kfac::spd_chol_pad(n);
  auto M = at::empty({cnt, N, N}, F.options());
  auto W = at::empty({cnt, N, N}, F.options());
  auto L = at::empty({cnt, N / 64, 64, 64}, F.options());
  kfac::spd_inverse_chol(F.data_ptr<float>(), X.data_ptr<float>(), M.data_ptr<float>(),
                         W.data_ptr<float>(), L.data_ptr<float>(), fail.data_ptr<int>(), n,
                         (int)cnt, (float)damping, s);
  return {X, fail};
}

// rocBLAS handle bound to stream s (shared with the two-stage eigensolver's
// strided GEMMs, csrc/twostage_host.cpp)
rocblas_handle kfac_rocblas_handle(hipStream_t s) { return handle_for(s).handle; }
