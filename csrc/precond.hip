// K-HIP-4 epilogue + K-HIP-7: eigen-basis scaling, KL-clip reduction and the
// in-place gradient write, all without host synchronisation.
//
// Reference behaviour:
//   eigen.py:370-384      v2 = v1 * dgda  or  v1 / (outer(dg, da) + damping)
//   base_preconditioner.py:409-433  vg = sum_l sum(P_l * grad_l) * lr^2,
//                         scale = 1 if vg == 0 else min(1, sqrt(kl / |vg|))
//                         -- two .item() host syncs PER LAYER in the
//                         reference; here one device-side double accumulator
//   layers/base.py:406-422 + modules.py:87-97  grad = scale * P, split into
//                         weight / bias grads (cat/split/contiguous in the
//                         reference; here written straight into .grad)
#include "common.h"

namespace kfac {

namespace {

inline unsigned grid_for(int64_t n, int64_t cap = 4096) {
  int64_t g = ceil_div(n, 256);
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}

__global__ void __launch_bounds__(256)
eigen_scale_kernel(float* __restrict__ v, int64_t rows, int64_t cols,
                   int64_t ldv, const float* __restrict__ dgda,
                   const float* __restrict__ dg, const float* __restrict__ da,
                   float damping) {
  const int64_t total = rows * cols;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += stride) {
    const int64_t i = e / cols, j = e - (e / cols) * cols;
    float x = v[i * ldv + j];
    if (dgda != nullptr) x *= dgda[e];
    else x /= (dg[i] * da[j] + damping);
    v[i * ldv + j] = x;
  }
}

template <typename TW, typename TB>
__global__ void __launch_bounds__(256)
kl_dot_kernel(const float* __restrict__ p, int64_t rows, int64_t cols,
              int64_t ldp, const TW* __restrict__ w, int64_t wcols,
              const TB* __restrict__ b, double* __restrict__ acc) {
  __shared__ double partial[4];
  double s = 0.0;
  const int64_t total = rows * cols;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += stride) {
    const int64_t i = e / cols, j = e - (e / cols) * cols;
    const float pv = p[i * ldp + j];
    float g;
    if (j < wcols) g = (float)w[i * wcols + j];
    else g = (float)b[i];
    s += (double)pv * (double)g;
  }
  s = wave_reduce_sum(s);
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) partial[wid] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double t = partial[0] + partial[1] + partial[2] + partial[3];
    if (t != 0.0) atomicAdd(acc, t);
  }
}

// scale = 1 if vg == 0 else min(1, sqrt(kl / |vg|)), vg = acc * lr^2.
// Resets the accumulator for the next step.
__global__ void kl_finalize_kernel(double* __restrict__ acc,
                                   float* __restrict__ scale, float kl_clip,
                                   float lr) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const double vg = acc[0] * (double)lr * (double)lr;
    double sc = 1.0;
    if (vg != 0.0) {
      sc = sqrt((double)kl_clip / fabs(vg));
      if (sc > 1.0) sc = 1.0;
    }
    scale[0] = (float)sc;
    acc[0] = 0.0;
  }
}

template <typename TW, typename TB>
__global__ void __launch_bounds__(256)
apply_grad_kernel(const float* __restrict__ p, int64_t rows, int64_t cols,
                  int64_t ldp, TW* __restrict__ w, int64_t wcols,
                  TB* __restrict__ b, const float* __restrict__ scale) {
  const float sc = scale != nullptr ? scale[0] : 1.f;
  const int64_t total = rows * cols;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += stride) {
    const int64_t i = e / cols, j = e - (e / cols) * cols;
    const float v = sc * p[i * ldp + j];
    if (j < wcols) w[i * wcols + j] = (TW)v;
    else b[i] = (TB)v;
  }
}

__global__ void __launch_bounds__(256)
identity_kernel(float* __restrict__ C, int64_t n, int64_t ldc) {
  const int64_t total = n * n;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += stride) {
    const int64_t i = e / n, j = e - (e / n) * n;
    C[i * ldc + j] = i == j ? 1.f : 0.f;
  }
}

}  // namespace

void eigen_scale(float* v, int64_t rows, int64_t cols, int64_t ldv,
                 const float* dgda, const float* dg, const float* da,
                 float damping, hipStream_t s) {
  const int64_t n = rows * cols;
  if (n == 0) return;
  eigen_scale_kernel<<<grid_for(n), 256, 0, s>>>(v, rows, cols, ldv, dgda, dg,
                                                 da, damping);
}

#define KFAC_DISPATCH_WB(WDT, BDT, MACRO)                                    \
  do {                                                                       \
    if ((WDT) == kF32 && (BDT) == kF32) MACRO(float, float);                 \
    else if ((WDT) == kBF16 && (BDT) == kBF16) MACRO(bf16_t, bf16_t);        \
    else if ((WDT) == kF16 && (BDT) == kF16) MACRO(__half, __half);          \
    else if ((WDT) == kF32) MACRO(float, bf16_t);                            \
    else MACRO(bf16_t, float);                                               \
  } while (0)

void kl_dot_accumulate(const float* p, int64_t rows, int64_t cols, int64_t ldp,
                       const void* wgrad, int wdtype, int64_t ldw,
                       const void* bgrad, int bdtype, double* acc,
                       hipStream_t s) {
  const int64_t n = rows * cols;
  if (n == 0) return;
  if (bgrad == nullptr) bdtype = wdtype;
#define KFAC_KL(TW, TB)                                                      \
  kl_dot_kernel<TW, TB><<<grid_for(n, 1024), 256, 0, s>>>(                   \
      p, rows, cols, ldp, (const TW*)wgrad, ldw, (const TB*)bgrad, acc)
  KFAC_DISPATCH_WB(wdtype, bdtype, KFAC_KL);
#undef KFAC_KL
}

void kl_scale_finalize(const double* acc, float* scale_out, float kl_clip,
                       float lr, hipStream_t s) {
  kl_finalize_kernel<<<1, 64, 0, s>>>(const_cast<double*>(acc), scale_out,
                                      kl_clip, lr);
}

void apply_grad(const float* p, int64_t rows, int64_t cols, int64_t ldp,
                void* wgrad, int wdtype, int64_t ldw, void* bgrad, int bdtype,
                const float* scale, hipStream_t s) {
  const int64_t n = rows * cols;
  if (n == 0) return;
  if (bgrad == nullptr) bdtype = wdtype;
#define KFAC_APPLY(TW, TB)                                                   \
  apply_grad_kernel<TW, TB><<<grid_for(n), 256, 0, s>>>(                     \
      p, rows, cols, ldp, (TW*)wgrad, ldw, (TB*)bgrad, scale)
  KFAC_DISPATCH_WB(wdtype, bdtype, KFAC_APPLY);
#undef KFAC_APPLY
}

void fill_identity_lerp(float* C, int64_t n, int64_t ldc, hipStream_t s) {
  if (n == 0) return;
  identity_kernel<<<grid_for(n * n), 256, 0, s>>>(C, n, ldc);
}

}  // namespace kfac
