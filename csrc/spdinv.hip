// K-HIP-5: batched damped SPD inverse  X = (F + damping I)^-1  for the
// K-FAC INVERSE method (reference kfac/layers/inverse.py:185-212 calls
// torch.linalg.inv once per factor, an LU with pivoting and a host sync for
// `info`).
//
// Small n (<= SPD_LDS_MAXN): one workgroup per matrix, the whole matrix
// resident in LDS, in-place Gauss-Jordan inversion without pivoting (the
// damped factor is SPD, so every pivot is positive and no row exchange is
// needed).  Per pivot k: stage row k / pivot and column k, then one fully
// parallel rank-1 update of the n x n LDS tile, then write the pivot row and
// column -- 2 barriers per pivot, no global memory traffic until the end.
// The result is written symmetrised, (X + X^T) / 2, so the triangle-packed
// broadcast (symmetry_aware) reproduces the inverse worker's copy exactly.

#include "common.h"

namespace kfac {

constexpr int SPD_LDS_MAXN = 176;  // (176 * 177 + 2 * 176) * 4 B = 126 KiB of LDS
constexpr int SPD_T = 512;

int spd_lds_max_n() { return SPD_LDS_MAXN; }

namespace {

__global__ void __launch_bounds__(SPD_T) spd_inverse_lds_kernel(
    const float* __restrict__ F, float* __restrict__ X, int n, int64_t strideF,
    int64_t strideX, float damping) {
  extern __shared__ float lds[];
  const int ld = n + 1;
  float* M = lds;               // [n][n+1]
  float* rowk = lds + n * ld;   // [n]
  float* colk = rowk + n;       // [n]
  const float* f = F + (int64_t)blockIdx.x * strideF;
  float* x = X + (int64_t)blockIdx.x * strideX;
  const int nn = n * n;
  for (int t = threadIdx.x; t < nn; t += SPD_T) {
    const int i = t / n, j = t - i * n;
    M[i * ld + j] = f[t] + (i == j ? damping : 0.f);
  }
  __syncthreads();
  for (int k = 0; k < n; ++k) {
    const float pinv = 1.f / M[k * ld + k];
    for (int t = threadIdx.x; t < n; t += SPD_T) {
      rowk[t] = M[k * ld + t] * pinv;
      colk[t] = M[t * ld + k];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < nn; t += SPD_T) {
      const int i = t / n, j = t - i * n;
      if (i == k) {
        M[i * ld + j] = (j == k) ? pinv : rowk[j];
      } else if (j == k) {
        M[i * ld + j] = -colk[i] * pinv;
      } else {
        M[i * ld + j] -= colk[i] * rowk[j];
      }
    }
    __syncthreads();
  }
  for (int t = threadIdx.x; t < nn; t += SPD_T) {
    const int i = t / n, j = t - i * n;
    x[t] = 0.5f * (M[i * ld + j] + M[j * ld + i]);
  }
}

}  // namespace

void spd_inverse_lds(const float* F, float* X, int n, int batch, int64_t strideF,
                     int64_t strideX, float damping, hipStream_t s) {
  if (batch <= 0 || n <= 0) return;
  const size_t shm = ((size_t)n * (n + 1) + 2 * (size_t)n) * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    const size_t maxshm =
        ((size_t)SPD_LDS_MAXN * (SPD_LDS_MAXN + 1) + 2 * (size_t)SPD_LDS_MAXN) * sizeof(float);
    KFAC_HIP_CHECK(hipFuncSetAttribute((const void*)spd_inverse_lds_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)maxshm));
    attr_set = true;
  }
  hipLaunchKernelGGL(spd_inverse_lds_kernel, dim3(batch), dim3(SPD_T), shm, s, F, X,
                     n, strideF, strideX, damping);
}

}  // namespace kfac
