// K-HIP-2 (stage 1): convolution patch extraction for the K-FAC A factor.
//
// Reference: Conv2dModuleHelper._extract_patches (kfac/layers/modules.py:
// 210-237) = pad + unfold x2 + transpose + contiguous, in (c, kh, kw) column
// order and fp32/whatever the activation dtype is.  Here:
//   * NHWC (channels_last) input -> rows (b, oy, ox), columns in the
//     "natural" (kh, kw, c) order.  Every (ky, kx) tap is a contiguous copy of
//     C channels, so the kernel moves 16-byte vectors end to end.  The K-FAC
//     layer keeps its A factor in this order and views the channels_last
//     weight gradient, whose physical layout is [out][kh][kw][c], with the
//     same column order -- no permutation anywhere on the hot path.
//   * NCHW input -> reference (c, kh, kw) order.
// Zero padding and stride are honoured; dilation / groups are rejected by
// the Python side (the reference silently ignores them).
#include "common.h"

namespace kfac {

namespace {

template <typename TI, typename TO>
__device__ __forceinline__ TO cvt(TI v) {
  return (TO)(float)v;
}
template <>
__device__ __forceinline__ float cvt<float, float>(float v) { return v; }
template <>
__device__ __forceinline__ bf16_t cvt<bf16_t, bf16_t>(bf16_t v) { return v; }

// scalar path: one thread per output element, c fastest (coalesced both ways)
template <typename TI, typename TO>
__global__ void __launch_bounds__(256)
im2col_nhwc_kernel(const TI* __restrict__ x, int64_t H, int64_t W, int64_t C,
                   int64_t sB, int64_t sH, int64_t sW, int kh, int kw, int sh,
                   int sw, int ph, int pw, int64_t OH, int64_t OW,
                   TO* __restrict__ out, int64_t ldo, int64_t total) {
  const int64_t KC = (int64_t)kh * kw * C;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += stride) {
    const int64_t row = e / KC;
    const int64_t col = e - row * KC;
    const int64_t tap = col / C;
    const int64_t c = col - tap * C;
    const int ky = (int)(tap / kw), kx = (int)(tap - (int64_t)(tap / kw) * kw);
    const int64_t b = row / (OH * OW);
    const int64_t rem = row - b * OH * OW;
    const int64_t oy = rem / OW, ox = rem - (rem / OW) * OW;
    const int64_t iy = oy * sh - ph + ky, ix = ox * sw - pw + kx;
    TO v = cvt<float, TO>(0.f);
    if (iy >= 0 && iy < H && ix >= 0 && ix < W)
      v = cvt<TI, TO>(x[b * sB + iy * sH + ix * sW + c]);
    out[row * ldo + col] = v;
  }
}

// vector path (same dtype in/out, C*sizeof % 16 == 0, aligned): one thread
// per 16-byte chunk of channels.
template <typename T>
__global__ void __launch_bounds__(256)
im2col_nhwc_vec_kernel(const T* __restrict__ x, int64_t H, int64_t W,
                       int64_t C, int64_t sB, int64_t sH, int64_t sW, int kh,
                       int kw, int sh, int sw, int ph, int pw, int64_t OH,
                       int64_t OW, T* __restrict__ out, int64_t ldo,
                       int64_t total_chunks) {
  constexpr int V = 16 / sizeof(T);
  const int64_t CC = C / V;             // chunks per tap
  const int64_t KCC = (int64_t)kh * kw * CC;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
       e < total_chunks; e += stride) {
    const int64_t row = e / KCC;
    const int64_t colc = e - row * KCC;
    const int64_t tap = colc / CC;
    const int64_t cc = colc - tap * CC;
    const int ky = (int)(tap / kw), kx = (int)(tap - (int64_t)(tap / kw) * kw);
    const int64_t b = row / (OH * OW);
    const int64_t rem = row - b * OH * OW;
    const int64_t oy = rem / OW, ox = rem - (rem / OW) * OW;
    const int64_t iy = oy * sh - ph + ky, ix = ox * sw - pw + kx;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (iy >= 0 && iy < H && ix >= 0 && ix < W)
      v = *reinterpret_cast<const uint4*>(x + b * sB + iy * sH + ix * sW +
                                          cc * V);
    *reinterpret_cast<uint4*>(out + row * ldo + tap * C + cc * V) = v;
  }
}

// NCHW -> reference (c, kh, kw) order; one thread per output element.
template <typename TI, typename TO>
__global__ void __launch_bounds__(256)
im2col_nchw_kernel(const TI* __restrict__ x, int64_t C, int64_t H, int64_t W,
                   int64_t sB, int64_t sC, int64_t sH, int64_t sW, int kh,
                   int kw, int sh, int sw, int ph, int pw, int64_t OH,
                   int64_t OW, TO* __restrict__ out, int64_t ldo,
                   int64_t total) {
  const int64_t KK = (int64_t)kh * kw;
  const int64_t KC = KK * C;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += stride) {
    const int64_t row = e / KC;
    const int64_t col = e - row * KC;
    const int64_t c = col / KK;
    const int64_t tap = col - c * KK;
    const int ky = (int)(tap / kw), kx = (int)(tap - (int64_t)(tap / kw) * kw);
    const int64_t b = row / (OH * OW);
    const int64_t rem = row - b * OH * OW;
    const int64_t oy = rem / OW, ox = rem - (rem / OW) * OW;
    const int64_t iy = oy * sh - ph + ky, ix = ox * sw - pw + kx;
    TO v = cvt<float, TO>(0.f);
    if (iy >= 0 && iy < H && ix >= 0 && ix < W)
      v = cvt<TI, TO>(x[b * sB + c * sC + iy * sH + ix * sW]);
    out[row * ldo + col] = v;
  }
}

// col2im, the adjoint of im2col_nhwc_vec_kernel (fp32, float4 lanes): gx[b][y][x][c] =
// sum over the taps (ky, kx) whose output pixel oy = (y + ph - ky) / sh, ox = (x + pw - kx) / sw
// is integral and in range of cols[(b, oy, ox)][(ky, kx, c)].  A strided convolution's input
// gradient as (dy . W) then col2im: every gx element is one thread's fixed-order sum, so the
// result is bit-reproducible (MIOpen's strided backward-data solvers are not).
__global__ void __launch_bounds__(256)
col2im_nhwc_kernel(const float4* __restrict__ cols, float4* __restrict__ gx, int64_t total4,
                   int C4, int H, int W, int OH, int OW, int kh, int kw, int sh, int sw, int ph,
                   int pw) {
  const int64_t KC4 = (int64_t)kh * kw * C4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total4;
       i += (int64_t)gridDim.x * 256) {
    const int64_t pix = i / C4;
    const int c = (int)(i - pix * C4);
    const int x = (int)(pix % W);
    const int64_t q = pix / W;
    const int y = (int)(q % H);
    const int64_t b = q / H;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int ky = 0; ky < kh; ++ky) {
      const int t = y + ph - ky;
      if (t < 0 || t % sh != 0 || t / sh >= OH) continue;
      const int64_t rowy = (b * OH + t / sh) * OW;
      for (int kx = 0; kx < kw; ++kx) {
        const int u = x + pw - kx;
        if (u < 0 || u % sw != 0 || u / sw >= OW) continue;
        const float4 v = cols[(rowy + u / sw) * KC4 + (int64_t)(ky * kw + kx) * C4 + c];
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
      }
    }
    gx[i] = a;
  }
}

// the bf16 variant (the bf16 autocast step's 3x3 input gradients, cols from a
// bf16 GEMM): 8 channels (16 bytes) per thread, summed in fp32 in the same
// fixed tap order, rounded once to bf16
__global__ void __launch_bounds__(256)
col2im_nhwc_bf16_kernel(const uint4* __restrict__ cols, uint4* __restrict__ gx, int64_t total8,
                        int C8, int H, int W, int OH, int OW, int kh, int kw, int sh, int sw,
                        int ph, int pw) {
  const int64_t KC8 = (int64_t)kh * kw * C8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total8;
       i += (int64_t)gridDim.x * 256) {
    const int64_t pix = i / C8;
    const int c = (int)(i - pix * C8);
    const int x = (int)(pix % W);
    const int64_t q = pix / W;
    const int y = (int)(q % H);
    const int64_t b = q / H;
    float a[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = 0.f;
    for (int ky = 0; ky < kh; ++ky) {
      const int t = y + ph - ky;
      if (t < 0 || t % sh != 0 || t / sh >= OH) continue;
      const int64_t rowy = (b * OH + t / sh) * OW;
      for (int kx = 0; kx < kw; ++kx) {
        const int u = x + pw - kx;
        if (u < 0 || u % sw != 0 || u / sw >= OW) continue;
        const uint4 v = cols[(rowy + u / sw) * KC8 + (int64_t)(ky * kw + kx) * C8 + c];
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[2 * e] += bf16_bits_to_f32((uint16_t)(w4[e] & 0xffffu));
          a[2 * e + 1] += bf16_bits_to_f32((uint16_t)(w4[e] >> 16));
        }
      }
    }
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      o[e] = (uint32_t)f32_to_bf16_bits(a[2 * e]) | ((uint32_t)f32_to_bf16_bits(a[2 * e + 1]) << 16);
    gx[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

inline unsigned grid_for(int64_t n) {
  int64_t g = ceil_div(n, 256);
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (unsigned)g;
}

template <typename TI, typename TO>
void nhwc_dispatch(const void* x, int64_t B, int64_t H, int64_t W, int64_t C,
                   int64_t sB, int64_t sH, int64_t sW, int kh, int kw, int sh,
                   int sw, int ph, int pw, int64_t OH, int64_t OW, void* out,
                   int64_t ldo, hipStream_t s) {
  const int64_t rows = B * OH * OW;
  if constexpr (std::is_same<TI, TO>::value) {
    constexpr int V = 16 / sizeof(TI);
    const bool ok =
        (C % V == 0) && (sB % V == 0) && (sH % V == 0) && (sW % V == 0) &&
        (ldo % V == 0) &&
        ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) &
         15) == 0;
    if (ok) {
      const int64_t chunks = rows * kh * kw * (C / V);
      im2col_nhwc_vec_kernel<TI><<<grid_for(chunks), 256, 0, s>>>(
          (const TI*)x, H, W, C, sB, sH, sW, kh, kw, sh, sw, ph, pw, OH, OW,
          (TI*)out, ldo, chunks);
      return;
    }
  }
  const int64_t total = rows * kh * kw * C;
  im2col_nhwc_kernel<TI, TO><<<grid_for(total), 256, 0, s>>>(
      (const TI*)x, H, W, C, sB, sH, sW, kh, kw, sh, sw, ph, pw, OH, OW,
      (TO*)out, ldo, total);
}

}  // namespace

void im2col_nhwc(int dtype, const void* x, int64_t B, int64_t H, int64_t W,
                 int64_t C, int64_t sB, int64_t sH, int64_t sW, int kh, int kw,
                 int sh, int sw, int ph, int pw, int64_t OH, int64_t OW,
                 void* out, int64_t ldo, int out_dtype, hipStream_t s) {
  if (B * OH * OW == 0) return;
#define KFAC_NHWC(TI, TO) \
  nhwc_dispatch<TI, TO>(x, B, H, W, C, sB, sH, sW, kh, kw, sh, sw, ph, pw, OH, OW, out, ldo, s)
  if (dtype == kBF16 && out_dtype == kBF16) KFAC_NHWC(bf16_t, bf16_t);
  else if (dtype == kF32 && out_dtype == kF32) KFAC_NHWC(float, float);
  else if (dtype == kF32 && out_dtype == kBF16) KFAC_NHWC(float, bf16_t);
  else if (dtype == kBF16 && out_dtype == kF32) KFAC_NHWC(bf16_t, float);
  else if (dtype == kF16 && out_dtype == kBF16) KFAC_NHWC(__half, bf16_t);
  else if (dtype == kF16 && out_dtype == kF32) KFAC_NHWC(__half, float);
#undef KFAC_NHWC
}

void im2col_nchw(int dtype, const void* x, int64_t B, int64_t C, int64_t H,
                 int64_t W, int64_t sB, int64_t sC, int64_t sH, int64_t sW,
                 int kh, int kw, int sh, int sw, int ph, int pw, int64_t OH,
                 int64_t OW, void* out, int64_t ldo, int out_dtype,
                 hipStream_t s) {
  const int64_t total = B * OH * OW * C * kh * kw;
  if (total == 0) return;
#define KFAC_NCHW(TI, TO)                                                     \
  im2col_nchw_kernel<TI, TO><<<grid_for(total), 256, 0, s>>>(                 \
      (const TI*)x, C, H, W, sB, sC, sH, sW, kh, kw, sh, sw, ph, pw, OH, OW,  \
      (TO*)out, ldo, total)
  if (dtype == kBF16 && out_dtype == kBF16) KFAC_NCHW(bf16_t, bf16_t);
  else if (dtype == kF32 && out_dtype == kF32) KFAC_NCHW(float, float);
  else if (dtype == kF32 && out_dtype == kBF16) KFAC_NCHW(float, bf16_t);
  else if (dtype == kBF16 && out_dtype == kF32) KFAC_NCHW(bf16_t, float);
  else if (dtype == kF16 && out_dtype == kBF16) KFAC_NCHW(__half, bf16_t);
  else if (dtype == kF16 && out_dtype == kF32) KFAC_NCHW(__half, float);
#undef KFAC_NCHW
}

void col2im_nhwc(int dtype, const void* cols, void* gx, int B, int H, int W, int C, int OH,
                 int OW, int kh, int kw, int sh, int sw, int ph, int pw, hipStream_t s) {
  if (dtype == kBF16) {
    const int64_t total8 = (int64_t)B * H * W * (C / 8);
    if (total8 == 0) return;
    col2im_nhwc_bf16_kernel<<<grid_for(total8), 256, 0, s>>>(
        (const uint4*)cols, (uint4*)gx, total8, C / 8, H, W, OH, OW, kh, kw, sh, sw, ph, pw);
    return;
  }
  const int64_t total4 = (int64_t)B * H * W * (C / 4);
  if (total4 == 0) return;
  col2im_nhwc_kernel<<<grid_for(total4), 256, 0, s>>>(
      (const float4*)cols, (float4*)gx, total4, C / 4, H, W, OH, OW, kh, kw, sh, sw, ph, pw);
}

}  // namespace kfac
