// Strided subsampling of NHWC activations and its adjoint, for the strided
// 1x1 projection convolutions (ops/conv.py _Subsample: conv(x[:, :, ::s,
// ::s]) as a stride-1 1x1 convolution of the subsampled input).
//
// Why: the adjoint is "zeros, then the gradient at every s-th pixel".  As a
// zero fill plus a strided TensorIterator copy it ran at 0.4 TB/s (118 us
// for ResNet-50's layer2 input at batch 32: profiles/r5/prof_fp32_r6z/).
// Here one pass writes every output element once, 16 bytes per thread,
// reading the gradient only at the kept pixels.
#include "common.h"

#include <cstdlib>

namespace kfac {

namespace {

// y[n][ho][wo][c] = x[n][ho * sh][wo * sw][c]; C % 4 == 0 (float4 lanes)
__global__ void __launch_bounds__(256) subsample_fwd_kernel(
    const float4* __restrict__ x, float4* __restrict__ y, int64_t total4, int C4, int H, int W,
    int Ho, int Wo, int sh, int sw) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total4;
       i += (int64_t)gridDim.x * 256) {
    const int64_t pix = i / C4;
    const int c = (int)(i - pix * C4);
    const int wo = (int)(pix % Wo);
    const int64_t q = pix / Wo;
    const int ho = (int)(q % Ho);
    const int64_t n = q / Ho;
    y[i] = x[((n * H + (int64_t)ho * sh) * W + (int64_t)wo * sw) * C4 + c];
  }
}

// gx[n][h][w][c] = (h % sh == 0 && w % sw == 0) ? g[n][h / sh][w / sw][c] : 0
__global__ void __launch_bounds__(256) subsample_bwd_kernel(
    const float4* __restrict__ g, float4* __restrict__ gx, int64_t total4, int C4, int H, int W,
    int Ho, int Wo, int sh, int sw) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total4;
       i += (int64_t)gridDim.x * 256) {
    const int64_t pix = i / C4;
    const int c = (int)(i - pix * C4);
    const int w = (int)(pix % W);
    const int64_t q = pix / W;
    const int h = (int)(q % H);
    const int64_t n = q / H;
    const int ho = h / sh, wo = w / sw;
    const bool kept = ho * sh == h && wo * sw == w && ho < Ho && wo < Wo;
    // the load is issued at a clamped in-bounds index and zeroed after
    const int64_t src = ((n * Ho + (kept ? ho : 0)) * Wo + (kept ? wo : 0)) * C4 + c;
    const float4 v = g[src];
    gx[i] = kept ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// gx[n][ho * sh][wo * sw][c] += g[n][ho][wo][c]: the adjoint accumulated
// into an existing full-size gradient (the other branch's), touching only
// the kept pixels
__global__ void __launch_bounds__(256) subsample_bwd_acc_kernel(
    const float4* __restrict__ g, float4* __restrict__ gx, int64_t total4, int C4, int H, int W,
    int Ho, int Wo, int sh, int sw) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total4;
       i += (int64_t)gridDim.x * 256) {
    const int64_t pix = i / C4;
    const int c = (int)(i - pix * C4);
    const int wo = (int)(pix % Wo);
    const int64_t q = pix / Wo;
    const int ho = (int)(q % Ho);
    const int64_t n = q / Ho;
    const int64_t dst = ((n * H + (int64_t)ho * sh) * W + (int64_t)wo * sw) * C4 + c;
    const float4 a = g[i], b = gx[dst];
    gx[dst] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
}

// y[p][0..C4) = x[p][0..C) zero-padded to a multiple of 4 channels, NHWC:
// one float4 of y per thread (the 3-channel stem input for the native
// weight gradient: one pass instead of a zero fill plus a cat)
__global__ void __launch_bounds__(256) pad_channels4_kernel(const float* __restrict__ x,
                                                            float4* __restrict__ y, int64_t total4,
                                                            int C, int C4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total4;
       i += (int64_t)gridDim.x * 256) {
    const int64_t pix = i / (C4 / 4);
    const int c0 = (int)(i - pix * (C4 / 4)) * 4;
    const float* px = x + pix * C;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = c0 + e < C ? px[c0 + e] : 0.f;
    y[i] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

int grid_for(int64_t total4) {
  const int64_t b = ceil_div(total4, 256);
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace

void subsample_fwd(const float* x, float* y, int N, int H, int W, int C, int sh, int sw,
                   hipStream_t s) {
  const int Ho = (H + sh - 1) / sh, Wo = (W + sw - 1) / sw;
  const int64_t total4 = (int64_t)N * Ho * Wo * (C / 4);
  if (total4 == 0) return;
  subsample_fwd_kernel<<<grid_for(total4), 256, 0, s>>>(
      (const float4*)x, (float4*)y, total4, C / 4, H, W, Ho, Wo, sh, sw);
}

void subsample_bwd(const float* g, float* gx, int N, int H, int W, int C, int sh, int sw,
                   hipStream_t s) {
  const int Ho = (H + sh - 1) / sh, Wo = (W + sw - 1) / sw;
  const int64_t total4 = (int64_t)N * H * W * (C / 4);
  if (total4 == 0) return;
  subsample_bwd_kernel<<<grid_for(total4), 256, 0, s>>>(
      (const float4*)g, (float4*)gx, total4, C / 4, H, W, Ho, Wo, sh, sw);
}

void pad_channels4(const float* x, float* y, int64_t pixels, int C, hipStream_t s) {
  const int C4 = (C + 3) / 4 * 4;
  const int64_t total4 = pixels * (C4 / 4);
  if (total4 == 0) return;
  pad_channels4_kernel<<<grid_for(total4), 256, 0, s>>>(x, (float4*)y, total4, C, C4);
}

void subsample_bwd_acc(const float* g, float* gx, int N, int H, int W, int C, int sh, int sw,
                       hipStream_t s) {
  const int Ho = (H + sh - 1) / sh, Wo = (W + sw - 1) / sw;
  const int64_t total4 = (int64_t)N * Ho * Wo * (C / 4);
  if (total4 == 0) return;
  subsample_bwd_acc_kernel<<<grid_for(total4), 256, 0, s>>>(
      (const float4*)g, (float4*)gx, total4, C / 4, H, W, Ho, Wo, sh, sw);
}

}  // namespace kfac

// ---- split-K partial sums: out[t] = sum_s part[s][t], s in fixed order
// (deterministic), float4 per thread.  torch's dim-0 reduction ran these at
// ~1 TB/s (617 us per ResNet-50 step over the native split-K convolutions,
// profiles/r5/prof_fp32_r6z/); this is one coalesced pass over the
// partials.  T % 4 == 0 and 16-byte aligned buffers (host checks).
namespace kfac {

namespace {

__global__ void __launch_bounds__(256) sum_splits_kernel(const float4* __restrict__ part,
                                                         float4* __restrict__ out, int S,
                                                         int64_t T4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < T4;
       i += (int64_t)gridDim.x * 256) {
    float4 a = part[i];
    // 4 partial loads in flight per step
    int s = 1;
    for (; s + 3 < S; s += 4) {
      const float4 b0 = part[(int64_t)s * T4 + i];
      const float4 b1 = part[(int64_t)(s + 1) * T4 + i];
      const float4 b2 = part[(int64_t)(s + 2) * T4 + i];
      const float4 b3 = part[(int64_t)(s + 3) * T4 + i];
      a.x += b0.x; a.y += b0.y; a.z += b0.z; a.w += b0.w;
      a.x += b1.x; a.y += b1.y; a.z += b1.z; a.w += b1.w;
      a.x += b2.x; a.y += b2.y; a.z += b2.z; a.w += b2.w;
      a.x += b3.x; a.y += b3.y; a.z += b3.z; a.w += b3.w;
    }
    for (; s < S; ++s) {
      const float4 b = part[(int64_t)s * T4 + i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    out[i] = a;
  }
}

// Few outputs, many splits (a small weight gradient split over many pixel
// blocks): G lanes per output float4 each sum every G-th partial, then the
// G lane sums are added in lane order through LDS -- fixed order for a
// given (S, T), so deterministic.  Thread t owns output e = t % E (E =
// 256 / G consecutive outputs: coalesced) and lane g = t / E.
template <int G>
__global__ void __launch_bounds__(256) sum_splits_grouped_kernel(const float4* __restrict__ part,
                                                                 float4* __restrict__ out, int S,
                                                                 int64_t T4) {
  constexpr int E = 256 / G;
  __shared__ float4 red[G][E];
  const int e = threadIdx.x % E, g = threadIdx.x / E;
  const int64_t i = (int64_t)blockIdx.x * E + e;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < T4) {
    int s = g;
    for (; s + 3 * G < S; s += 4 * G) {
      const float4 b0 = part[(int64_t)s * T4 + i];
      const float4 b1 = part[(int64_t)(s + G) * T4 + i];
      const float4 b2 = part[(int64_t)(s + 2 * G) * T4 + i];
      const float4 b3 = part[(int64_t)(s + 3 * G) * T4 + i];
      a.x += b0.x; a.y += b0.y; a.z += b0.z; a.w += b0.w;
      a.x += b1.x; a.y += b1.y; a.z += b1.z; a.w += b1.w;
      a.x += b2.x; a.y += b2.y; a.z += b2.z; a.w += b2.w;
      a.x += b3.x; a.y += b3.y; a.z += b3.z; a.w += b3.w;
    }
    for (; s < S; s += G) {
      const float4 b = part[(int64_t)s * T4 + i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
  }
  red[g][e] = a;
  __syncthreads();
  if (g == 0 && i < T4) {
#pragma unroll 4
    for (int q = 1; q < G; ++q) {
      const float4 b = red[q][e];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    out[i] = a;
  }
}

}  // namespace

void sum_splits(const float* part, float* out, int S, int64_t T, hipStream_t s) {
  const int64_t T4 = T / 4;
  if (T4 == 0 || S <= 0) return;
  // lanes per output: enough threads to cover ~64K with at least 4
  // partials per lane
  static const int gmax = [] {
    const char* e = std::getenv("KFAC_SUM_SPLITS_GROUP");
    return e != nullptr ? std::atoi(e) : 16;
  }();
  int G = 1;
  while (G < gmax && T4 * G < 65536 && 4 * (2 * G) <= S) G *= 2;
#define KFAC_SSG(GV)                                                                    \
  sum_splits_grouped_kernel<GV><<<(unsigned)ceil_div(T4, 256 / GV), 256, 0, s>>>(       \
      (const float4*)part, (float4*)out, S, T4)
  if (G >= 16) { KFAC_SSG(16); return; }
  if (G == 8) { KFAC_SSG(8); return; }
  if (G == 4) { KFAC_SSG(4); return; }
  if (G == 2) { KFAC_SSG(2); return; }
#undef KFAC_SSG
  int64_t b = ceil_div(T4, 256);
  if (b > 4096) b = 4096;
  sum_splits_kernel<<<(unsigned)b, 256, 0, s>>>((const float4*)part, (float4*)out, S, T4);
}

}  // namespace kfac
