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

}  // namespace kfac
