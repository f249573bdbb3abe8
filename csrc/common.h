// Shared helpers for the MI355X (gfx950) K-FAC kernels.
//
// Kernel translation units (*.hip) include only this header and the HIP
// runtime; they export plain C++ launchers taking raw device pointers and a
// hipStream_t.  bindings.cpp is the only file that sees torch/ATen.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <cstdint>
#include <cstdio>

#define KFAC_HIP_CHECK(expr)                                                   \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e),        \
              __FILE__, __LINE__);                                             \
    }                                                                          \
  } while (0)

namespace kfac {

// dtype tags shared with bindings.cpp
enum DType : int { kF32 = 0, kBF16 = 1, kF64 = 2, kF16 = 3 };

using bf16_t = __hip_bfloat16;

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(double x) { return (float)x; }
__device__ __forceinline__ float to_f32(bf16_t x) { return __bfloat162float(x); }
__device__ __forceinline__ float to_f32(__half x) { return __half2float(x); }

__device__ __forceinline__ float bf16_bits_to_f32(uint16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}

// round-to-nearest-even fp32 -> bf16 bits (no NaN special-casing needed for
// finite K-FAC activations, but NaN is preserved as a quiet NaN)
__device__ __forceinline__ uint16_t f32_to_bf16_bits(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) {
    return (uint16_t)((u >> 16) | 0x40);
  }
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) {
  return (a + b - 1) / b;
}

__device__ __forceinline__ float wave_reduce_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Full-wave float sum, returned wave-uniform, with no LDS round trip: DPP
// quad / half-row / row mirrors leave every lane with its 16-lane row sum,
// then the four row sums are read out with v_readlane.  ds_bpermute-based
// __shfl_xor reductions cost an LDS round trip per step, and the compiler
// does not overlap independent ones (sytrd col step: 65 reductions, 12 us).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, true));
}

__device__ __forceinline__ float wave_sum_uniform(float v) {
  v += dpp_mov<0xb1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_mov<0x4e>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  const int b = __builtin_bit_cast(int, v);
  return (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16))) +
         (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48)));
}

__device__ __forceinline__ double wave_reduce_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

}  // namespace kfac
