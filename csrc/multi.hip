// K-HIP-7 (multi-tensor form): the KL-clip reduction and the scaled gradient
// write for ALL layers of a step in one launch each.
//
// The reference does, per layer, two `.item()` host syncs plus a cat/split/
// contiguous chain (base_preconditioner.py:409-433, layers/base.py:406-422).
// ResNet-50 has 54 K-FAC layers: one launch per layer per op is ~110 small
// launches per step on the critical path.  Here a step issues three:
//   kl_dot_multi    part[b] = block b's share of sum_l <P_l, [Wg_l | bg_l]>
//   kl_finalize_dev scale = min(1, sqrt(kl_clip / |sum_b part[b] * lr^2|))
// The per-block fp64 partials are summed in a fixed order (no atomics), so
// the KL-clip scale -- and every gradient it multiplies -- is bitwise
// reproducible run to run and between graph replay and eager execution.
//   apply_multi     [Wg_l | bg_l] = scale * P_l
// Under tensor parallelism kl_reduce_partials folds the partials into one
// per-rank sum that a single all-reduce over the model-parallel group
// combines before kl_finalize_dev (nparts = 1).
// Layers are described by a device-resident descriptor table; each block
// finds its layer by binary search over the per-layer block prefix sums.
// kl_clip and lr are read from a small device array so the launches can be
// captured in a HIP graph and replayed with new hyperparameters.
#include "common.h"
#include "descs.h"

namespace kfac {


namespace {

constexpr int MT = 256;
constexpr int EPT = 8;  // elements per thread per block
constexpr int KL_RED = 256;  // threads of the partial-sum reduction

// The table's pointers are generic to the compiler; address-space-1 casts
// make the accesses global_load/store instead of FLAT (which also count on
// lgkmcnt).
#define GLOBAL __attribute__((address_space(1)))

__device__ __forceinline__ float load_any(const void* base, int64_t i, int dt) {
  if (dt == kF32) return ((const GLOBAL float*)base)[i];
  const unsigned short u = ((const GLOBAL unsigned short*)base)[i];
  if (dt == kBF16) return __uint_as_float((uint32_t)u << 16);
  return __half2float(__ushort_as_half(u));
}

__device__ __forceinline__ void store_any(void* base, int64_t i, int dt, float v) {
  if (dt == kF32) {
    ((GLOBAL float*)base)[i] = v;
    return;
  }
  const unsigned short u = dt == kBF16 ? __bfloat16_as_ushort(__float2bfloat16(v))
                                       : __half_as_ushort(__float2half(v));
  ((GLOBAL unsigned short*)base)[i] = u;
}

__device__ __forceinline__ float load_p(const float* p, int64_t i) {
  return ((const GLOBAL float*)p)[i];
}

__device__ __forceinline__ int find_layer(const LayerDesc* d, int n, int64_t blk) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].block_start <= blk) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ void __launch_bounds__(MT)
kl_dot_multi_kernel(const LayerDesc* __restrict__ descs, int nlayers,
                    double* __restrict__ acc) {
  __shared__ double part[MT / 64];
  const int li = find_layer(descs, nlayers, blockIdx.x);
  const LayerDesc d = descs[li];
  const int64_t total = d.rows * d.cols;
  const int64_t base = (int64_t)(blockIdx.x - d.block_start) * MT * EPT;
  // every load of the thread first (clamped in-bounds elements, masked in
  // the sum): one memory round trip, not one per element
  float pv[EPT], gv[EPT];
  uint32_t ii[EPT], jj[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int64_t e = base + k * MT + threadIdx.x;
    const uint32_t ue = (uint32_t)(e < total ? e : 0), uc = (uint32_t)d.cols;
    ii[k] = ue / uc;
    jj[k] = ue - ii[k] * uc;
    pv[k] = load_p(d.p, (int64_t)ii[k] * d.ldp + jj[k]);
  }
  // gradient element (weight column, or the bias column scaled by bscale);
  // the dtype branch is uniform, outside the element loop
#define KFAC_G_SRC(k) (jj[k] < (uint32_t)d.wcols ? d.w : d.b)
#define KFAC_G_IDX(k) (jj[k] < (uint32_t)d.wcols ? (int64_t)ii[k] * d.wcols + jj[k] : (int64_t)ii[k])
#define KFAC_G_SC(k) (jj[k] < (uint32_t)d.wcols ? 1.f : d.bscale)
  if ((d.b == nullptr || d.bdt == d.wdt) && d.wdt == kF32) {
#pragma unroll
    for (int k = 0; k < EPT; ++k)
      gv[k] = ((const GLOBAL float*)KFAC_G_SRC(k))[KFAC_G_IDX(k)] * KFAC_G_SC(k);
  } else if (d.b == nullptr || d.bdt == d.wdt) {
    unsigned short u[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) u[k] = ((const GLOBAL unsigned short*)KFAC_G_SRC(k))[KFAC_G_IDX(k)];
#pragma unroll
    for (int k = 0; k < EPT; ++k)
      gv[k] = (d.wdt == kBF16 ? __uint_as_float((uint32_t)u[k] << 16)
                              : __half2float(__ushort_as_half(u[k]))) * KFAC_G_SC(k);
  } else {
#pragma unroll
    for (int k = 0; k < EPT; ++k)
      gv[k] = load_any(KFAC_G_SRC(k), KFAC_G_IDX(k),
                       jj[k] < (uint32_t)d.wcols ? d.wdt : d.bdt) * KFAC_G_SC(k);
  }
#undef KFAC_G_SRC
#undef KFAC_G_IDX
#undef KFAC_G_SC
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < EPT; ++k)
    if (base + k * MT + threadIdx.x < total) s += (double)pv[k] * (double)gv[k];
  s = wave_reduce_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < MT / 64; ++w) t += part[w];
    acc[blockIdx.x] = t;  // one slot per block: no atomics, fixed order
  }
}

// params: [0] kl_clip, [1] lr.  acc: nparts per-block partial sums.
__global__ void __launch_bounds__(KL_RED)
kl_finalize_dev_kernel(const double* __restrict__ acc, int64_t nparts,
                       const float* __restrict__ params, float* __restrict__ scale) {
  __shared__ double part[KL_RED / 64];
  double v = 0.0;
  for (int64_t i = threadIdx.x; i < nparts; i += KL_RED) v += acc[i];
  v = wave_reduce_sum(v);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < KL_RED / 64; ++w) tot += part[w];
    const double lr = params[1];
    const double vg = tot * lr * lr;
    double sc = 1.0;
    if (vg != 0.0) {
      sc = sqrt((double)params[0] / fabs(vg));
      if (sc > 1.0) sc = 1.0;
    }
    scale[0] = (float)sc;
  }
}

// out[0] = sum of the nparts partials in a fixed order (the per-rank KL sum
// that a model-parallel all-reduce combines before kl_finalize_dev)
__global__ void __launch_bounds__(KL_RED)
kl_reduce_partials_kernel(const double* __restrict__ acc, int64_t nparts,
                          double* __restrict__ out) {
  __shared__ double part[KL_RED / 64];
  double v = 0.0;
  for (int64_t i = threadIdx.x; i < nparts; i += KL_RED) v += acc[i];
  v = wave_reduce_sum(v);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < KL_RED / 64; ++w) tot += part[w];
    out[0] = tot;
  }
}

__global__ void __launch_bounds__(MT)
apply_multi_kernel(const LayerDesc* __restrict__ descs, int nlayers,
                   const float* __restrict__ scale) {
  const int li = find_layer(descs, nlayers, blockIdx.x);
  const LayerDesc d = descs[li];
  const float sc = scale != nullptr ? scale[0] : 1.f;
  const int64_t total = d.rows * d.cols;
  const int64_t base = (int64_t)(blockIdx.x - d.block_start) * MT * EPT;
  // loads first (clamped), then the stores
  float pv[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int64_t e = base + k * MT + threadIdx.x;
    const uint32_t ue = (uint32_t)(e < total ? e : 0), uc = (uint32_t)d.cols;
    const uint32_t i = ue / uc, j = ue - i * uc;
    pv[k] = load_p(d.p, (int64_t)i * d.ldp + j);
  }
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int64_t e = base + k * MT + threadIdx.x;
    if (e < total) {
      const uint32_t ue = (uint32_t)e, uc = (uint32_t)d.cols;
      const uint32_t i = ue / uc, j = ue - i * uc;
      const float v = sc * pv[k];
      if (j < d.wcols) store_any(d.w, (int64_t)i * d.wcols + j, d.wdt, v);
      else store_any(d.b, i, d.bdt, v);
    }
  }
}

}  // namespace

int64_t multi_blocks_for(int64_t rows, int64_t cols) {
  return ceil_div(rows * cols, (int64_t)MT * EPT);
}

void kl_dot_multi(const LayerDesc* descs, int nlayers, int64_t total_blocks,
                  double* acc, hipStream_t s) {
  if (nlayers == 0 || total_blocks == 0) return;
  kl_dot_multi_kernel<<<dim3((unsigned)total_blocks), dim3(MT), 0, s>>>(
      descs, nlayers, acc);
}

void kl_finalize_dev(const double* acc, int64_t nparts, const float* params,
                     float* scale, hipStream_t s) {
  kl_finalize_dev_kernel<<<1, KL_RED, 0, s>>>(acc, nparts, params, scale);
}

void kl_reduce_partials(const double* acc, int64_t nparts, double* out, hipStream_t s) {
  kl_reduce_partials_kernel<<<1, KL_RED, 0, s>>>(acc, nparts, out);
}

void apply_multi(const LayerDesc* descs, int nlayers, int64_t total_blocks,
                 const float* scale, hipStream_t s) {
  if (nlayers == 0 || total_blocks == 0) return;
  apply_multi_kernel<<<dim3((unsigned)total_blocks), dim3(MT), 0, s>>>(
      descs, nlayers, scale);
}

}  // namespace kfac
