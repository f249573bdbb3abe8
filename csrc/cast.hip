// Multi-tensor fp32 <-> bf16 cast: every conv / linear weight of a model in
// ONE launch (forward: fp32 master weights -> bf16 compute copies) and every
// weight gradient in one launch back (bf16 -> fp32).
//
// Why: under bf16 autocast PyTorch casts each weight separately on every
// forward and each weight gradient separately on every backward.  In a
// graph-replayed ResNet-50 step at batch 32 that is 57 + 56 tiny kernels,
// ~4.9 us each, ~0.55 ms of a ~8.6 ms SGD step
// (profiles/step_kernel_diff_resnet50_r2.txt), for ~150 MB of traffic that
// one launch streams in ~30 us.  Rounding is round-to-nearest-even, as
// torch's cast.
#include "common.h"
#include "descs.h"

namespace kfac {

namespace {

constexpr int CT = 256;   // threads per block
constexpr int CE = 8;     // elements per thread
#define GLOBAL __attribute__((address_space(1)))
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int find_cast(const CastDesc* d, int n, int64_t blk) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].block_start <= blk) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

template <bool TO_BF16>
__global__ void __launch_bounds__(CT) cast_multi_kernel(const CastDesc* __restrict__ descs, int nd) {
  const CastDesc d = descs[find_cast(descs, nd, blockIdx.x)];
  const int64_t e0 = ((int64_t)(blockIdx.x - d.block_start) * CT + threadIdx.x) * CE;
  if (e0 >= d.n) return;
  const bool full = d.vec && e0 + CE <= d.n;
  if constexpr (TO_BF16) {
    const GLOBAL float* s = (const GLOBAL float*)d.src + e0;
    GLOBAL uint16_t* o = (GLOBAL uint16_t*)d.dst + e0;
    if (full) {
      const f4_t a = *(const GLOBAL f4_t*)s;
      const f4_t b = *(const GLOBAL f4_t*)(s + 4);
      u4_t u;
      u.x = (uint32_t)f32_to_bf16_bits(a.x) | ((uint32_t)f32_to_bf16_bits(a.y) << 16);
      u.y = (uint32_t)f32_to_bf16_bits(a.z) | ((uint32_t)f32_to_bf16_bits(a.w) << 16);
      u.z = (uint32_t)f32_to_bf16_bits(b.x) | ((uint32_t)f32_to_bf16_bits(b.y) << 16);
      u.w = (uint32_t)f32_to_bf16_bits(b.z) | ((uint32_t)f32_to_bf16_bits(b.w) << 16);
      *(GLOBAL u4_t*)o = u;
    } else {
      for (int e = 0; e < CE && e0 + e < d.n; ++e) o[e] = f32_to_bf16_bits(s[e]);
    }
  } else {
    const GLOBAL uint16_t* s = (const GLOBAL uint16_t*)d.src + e0;
    GLOBAL float* o = (GLOBAL float*)d.dst + e0;
    if (full) {
      const u4_t u = *(const GLOBAL u4_t*)s;
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
      f4_t a, b;
      a.x = __uint_as_float(w[0] << 16);
      a.y = __uint_as_float(w[0] & 0xffff0000u);
      a.z = __uint_as_float(w[1] << 16);
      a.w = __uint_as_float(w[1] & 0xffff0000u);
      b.x = __uint_as_float(w[2] << 16);
      b.y = __uint_as_float(w[2] & 0xffff0000u);
      b.z = __uint_as_float(w[3] << 16);
      b.w = __uint_as_float(w[3] & 0xffff0000u);
      *(GLOBAL f4_t*)o = a;
      *(GLOBAL f4_t*)(o + 4) = b;
    } else {
      for (int e = 0; e < CE && e0 + e < d.n; ++e) o[e] = __uint_as_float((uint32_t)s[e] << 16);
    }
  }
}

}  // namespace

int64_t cast_blocks_for(int64_t n) { return ceil_div(n, (int64_t)CT * CE); }

void cast_multi(const CastDesc* table, int n, int64_t total_blocks, bool to_bf16,
                hipStream_t s) {
  if (n <= 0 || total_blocks <= 0) return;
  if (to_bf16)
    cast_multi_kernel<true><<<dim3((unsigned)total_blocks), dim3(CT), 0, s>>>(table, n);
  else
    cast_multi_kernel<false><<<dim3((unsigned)total_blocks), dim3(CT), 0, s>>>(table, n);
}

}  // namespace kfac
