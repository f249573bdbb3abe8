// K-HIP-6: symmetric (upper-triangle) pack / unpack and scaled copies for the
// K-FAC communication buckets (reference: get_triu / fill_triu in
// kfac/distributed.py:416-459, and the 1/world average in the all-reduce
// callbacks, :226-240).
//
// Layout of a packed triangle: row-major upper triangle including the
// diagonal, i.e. element (i, j>=i) of an n x n matrix lives at
//   off(i) + (j - i),  off(i) = i*n - i*(i-1)/2.
// This is exactly torch.triu_indices order, so buffers are interchangeable
// with the reference's packed format.
#include "common.h"

namespace kfac {

__host__ __device__ inline int64_t triu_row_offset(int64_t i, int64_t n) {
  return i * n - (i * (i - 1)) / 2;
}

// one block per row: coalesced read of src row i (cols i..n-1), coalesced
// write to the packed row.
template <typename T>
__global__ void __launch_bounds__(256)
triu_pack_kernel(const T* __restrict__ src, int64_t ld, int64_t n,
                 T* __restrict__ dst) {
  const int64_t i = blockIdx.x;
  const int64_t base = triu_row_offset(i, n);
  const T* row = src + i * ld;
  for (int64_t j = i + threadIdx.x; j < n; j += blockDim.x) {
    dst[base + (j - i)] = row[j];
  }
}

// 32x32 tiles over the full output.  Upper (and diagonal) tiles copy from the
// packed rows directly; lower tiles stage the mirrored upper tile through LDS
// and write it transposed, so both the packed reads and the dense writes stay
// coalesced.  dst = scale * symmetric(packed).
template <typename T>
__global__ void __launch_bounds__(256)
triu_unpack_kernel(const T* __restrict__ packed, int64_t n, T* __restrict__ dst,
                   int64_t ld, float scale) {
  __shared__ T tile[32][33];
  const int64_t ti = blockIdx.y, tj = blockIdx.x;  // tile row, tile col
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  if (ti <= tj) {
    for (int r = ty; r < 32; r += 8) {
      const int64_t i = ti * 32 + r, j = tj * 32 + tx;
      if (i < n && j < n) {
        T v;
        if (j >= i) {
          v = packed[triu_row_offset(i, n) + (j - i)];
        } else {  // only inside diagonal tiles
          v = packed[triu_row_offset(j, n) + (i - j)];
        }
        dst[i * ld + j] = (T)((float)v * scale);
      }
    }
  } else {
    // read upper tile (tj, ti): rows tj*32.., cols ti*32.. (all cols > rows)
    for (int r = ty; r < 32; r += 8) {
      const int64_t i = tj * 32 + r, j = ti * 32 + tx;
      if (i < n && j < n) tile[r][tx] = packed[triu_row_offset(i, n) + (j - i)];
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
      const int64_t i = ti * 32 + r, j = tj * 32 + tx;
      if (i < n && j < n) dst[i * ld + j] = (T)((float)tile[tx][r] * scale);
    }
  }
}

// dst[k] = scale * src[k] (vectorised by 4 when aligned)
template <typename T>
__global__ void __launch_bounds__(256)
scale_copy_kernel(const T* __restrict__ src, T* __restrict__ dst, int64_t n,
                  float scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += stride) {
    dst[k] = (T)((float)src[k] * scale);
  }
}

template <>
__global__ void __launch_bounds__(256)
scale_copy_kernel<float>(const float* __restrict__ src, float* __restrict__ dst,
                         int64_t n, float scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = ((reinterpret_cast<uintptr_t>(src) |
                       reinterpret_cast<uintptr_t>(dst)) & 15) == 0 ? n / 4 : 0;
  const float4* s4 = reinterpret_cast<const float4*>(src);
  float4* d4 = reinterpret_cast<float4*>(dst);
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n4;
       k += stride) {
    float4 v = s4[k];
    v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
    d4[k] = v;
  }
  for (int64_t k = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
       k < n; k += stride) {
    dst[k] = src[k] * scale;
  }
}

static inline int grid_for(int64_t n) {
  int64_t g = ceil_div(n, 256);
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

template <typename T>
static void launch_pack(const void* src, int64_t ld, int64_t n, void* dst,
                        hipStream_t s) {
  if (n <= 0) return;
  triu_pack_kernel<T><<<dim3((unsigned)n), dim3(256), 0, s>>>(
      (const T*)src, ld, n, (T*)dst);
}

template <typename T>
static void launch_unpack(const void* packed, int64_t n, void* dst, int64_t ld,
                          float scale, hipStream_t s) {
  if (n <= 0) return;
  const unsigned t = (unsigned)ceil_div(n, 32);
  triu_unpack_kernel<T><<<dim3(t, t), dim3(256), 0, s>>>(
      (const T*)packed, n, (T*)dst, ld, scale);
}

void triu_pack(int dtype, const void* src, int64_t ld, int64_t n, void* dst,
               hipStream_t s) {
  if (dtype == kF32) launch_pack<float>(src, ld, n, dst, s);
  else if (dtype == kF64) launch_pack<double>(src, ld, n, dst, s);
  else launch_pack<bf16_t>(src, ld, n, dst, s);
}

void triu_unpack(int dtype, const void* packed, int64_t n, void* dst,
                 int64_t ld, float scale, hipStream_t s) {
  if (dtype == kF32) launch_unpack<float>(packed, n, dst, ld, scale, s);
  else if (dtype == kF64) launch_unpack<double>(packed, n, dst, ld, scale, s);
  else launch_unpack<bf16_t>(packed, n, dst, ld, scale, s);
}

void scale_copy(int dtype, const void* src, void* dst, int64_t n, float scale,
                hipStream_t s) {
  if (n <= 0) return;
  const int g = grid_for(dtype == kF32 ? ceil_div(n, 4) : n);
  if (dtype == kF32)
    scale_copy_kernel<float><<<g, 256, 0, s>>>((const float*)src, (float*)dst, n, scale);
  else if (dtype == kF64)
    scale_copy_kernel<double><<<g, 256, 0, s>>>((const double*)src, (double*)dst, n, scale);
  else
    scale_copy_kernel<bf16_t><<<g, 256, 0, s>>>((const bf16_t*)src, (bf16_t*)dst, n, scale);
}

}  // namespace kfac
