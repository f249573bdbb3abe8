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

__device__ __forceinline__ double wave_reduce_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

}  // namespace kfac
