// 64x64x64 fp32 MFMA tile product on LDS operands, used by the blocked SPD
// inverse (spdinv_chol.hip).
//
// A 256-thread block = 4 waves; wave w computes the 32x32 quadrant
// (wi, wj) = (w >> 1, w & 1) of  C = A^T * Bt  with both operands stored
// k-major in LDS (A as [k][i], Bt as [k][j], row stride TILE_LD floats), so
// each half-wave reads 32 consecutive floats (conflict-free) per MFMA.
// v_mfma_f32_32x32x2_f32: exact fp32 products (no TF32 on gfx950), lane l
// holds A[i = l & 31][k = l >> 5] and B[k = l >> 5][j = l & 31]; C/D:
// col = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5).
#pragma once

#include <hip/hip_runtime.h>

namespace kfac {
namespace tile {

constexpr int T64 = 64;
constexpr int TILE_LD = T64 + 4;  // 68 floats: 16-B aligned rows

typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ v16f mm64(const float* A, const float* Bt, int wi, int wj) {
  const int l = threadIdx.x & 63;
  const int r = l & 31, h = l >> 5;
  v16f acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll 8
  for (int k = 0; k < T64; k += 2) {
    const float av = A[(k + h) * TILE_LD + wi * 32 + r];
    const float bv = Bt[(k + h) * TILE_LD + wj * 32 + r];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
  }
  return acc;
}

// acc += A^T * Bt (same operand layout as mm64)
__device__ __forceinline__ v16f mm64_acc(const float* A, const float* Bt, int wi, int wj,
                                         v16f acc) {
  const int l = threadIdx.x & 63;
  const int r = l & 31, h = l >> 5;
#pragma unroll 8
  for (int k = 0; k < T64; k += 2) {
    const float av = A[(k + h) * TILE_LD + wi * 32 + r];
    const float bv = Bt[(k + h) * TILE_LD + wj * 32 + r];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
  }
  return acc;
}

// a wave's 32x32 accumulator quadrant -> LDS tile T[i][j] (TRANS: T[j][i])
template <bool TRANS>
__device__ __forceinline__ void store_quad(float* T, const v16f& acc, int wi, int wj) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int row = wi * 32 + (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
    const int col = wj * 32 + (l & 31);
    if (TRANS) T[col * TILE_LD + row] = acc[e];
    else T[row * TILE_LD + col] = acc[e];
  }
}

// global [64][64] block (row stride ld) -> LDS, natural ([i][j]) or
// transposed ([j][i]); 256 threads, float4 global loads
template <bool TRANS>
__device__ __forceinline__ void load64(float* T, const float* g, int64_t ld) {
  for (int e = threadIdx.x; e < T64 * (T64 / 4); e += 256) {
    const int i = e >> 4, c4 = (e & 15) * 4;
    const float4 v = *reinterpret_cast<const float4*>(g + (int64_t)i * ld + c4);
    if (TRANS) {
      T[(c4 + 0) * TILE_LD + i] = v.x;
      T[(c4 + 1) * TILE_LD + i] = v.y;
      T[(c4 + 2) * TILE_LD + i] = v.z;
      T[(c4 + 3) * TILE_LD + i] = v.w;
    } else {
      *reinterpret_cast<float4*>(&T[i * TILE_LD + c4]) = v;
    }
  }
}

// LDS [64][64] natural tile -> global block (row stride ld), scaled
__device__ __forceinline__ void store64(float* g, int64_t ld, const float* T, float scale) {
  for (int e = threadIdx.x; e < T64 * (T64 / 4); e += 256) {
    const int i = e >> 4, c4 = (e & 15) * 4;
    float4 v = *reinterpret_cast<const float4*>(&T[i * TILE_LD + c4]);
    v.x *= scale;
    v.y *= scale;
    v.z *= scale;
    v.w *= scale;
    *reinterpret_cast<float4*>(g + (int64_t)i * ld + c4) = v;
  }
}

}  // namespace tile
}  // namespace kfac
