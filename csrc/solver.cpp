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

#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

struct HandleState {
  rocblas_handle handle = nullptr;
  at::Tensor workspace;
};

std::mutex g_mu;
std::unordered_map<hipStream_t, HandleState> g_handles;

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
