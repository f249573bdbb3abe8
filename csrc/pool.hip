// Max pooling of NHWC (channels_last) activations with a one-byte argmax
// code, and its adjoint as a gather (ops/pool.py MaxPool2dNHWC; ResNet's
// 3x3 / stride-2 stem pool).
//
// Why: torch's NHWC max_pool2d stores int64 indices (8 bytes per output
// element) and its backward ran 83 us per ResNet-50 step at batch 32 for a
// 103 MB input gradient (profiles/r6/prof_r8/).  Here the forward stores the
// window position (kh * kw_size + kw, < 256) as one byte, and the backward
// has each thread own 4 (fp32) or 8 (bf16) channels of one input pixel:
// it visits the <= ceil(k/s)^2 windows that contain the pixel, in a fixed
// order, and adds the gradient of those whose code points at it -- every
// input-gradient element written once, no atomics, bit-reproducible.
//
// Semantics follow torch.nn.functional.max_pool2d (dilation 1, no ceil
// mode): padding is never a candidate, the first maximum in row-major window
// order wins, NaN propagates (a NaN takes over wherever it appears).
#include "common.h"

namespace kfac {

namespace {

template <typename E> struct Vec;
template <> struct Vec<float> {
  static constexpr int N = 4;
  __device__ __forceinline__ static void load(const float* p, float* v) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
  __device__ __forceinline__ static void store(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct Vec<uint16_t> {  // bf16 bits
  static constexpr int N = 8;
  __device__ __forceinline__ static void load(const uint16_t* p, float* v) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void store(uint16_t* p, const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = (uint32_t)f32_to_bf16_bits(v[2 * i]) |
             ((uint32_t)f32_to_bf16_bits(v[2 * i + 1]) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};

struct PoolGeom {
  int H, W, C, OH, OW, k, s, p;
};

template <typename E>
__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const E* __restrict__ x,
                                                          E* __restrict__ y,
                                                          uint8_t* __restrict__ code,
                                                          int64_t total, PoolGeom g) {
  constexpr int V = Vec<E>::N;
  const int CV = g.C / V;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    const int cv = (int)(i % CV);
    const int64_t pix = i / CV;
    const int ow = (int)(pix % g.OW);
    const int64_t q = pix / g.OW;
    const int oh = (int)(q % g.OH);
    const int64_t n = q / g.OH;
    float m[V];
    int best[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      m[e] = -__builtin_inff();
      best[e] = 0;
    }
    bool any = false;
    for (int kh = 0; kh < g.k; ++kh) {
      const int h = oh * g.s - g.p + kh;
      if ((unsigned)h >= (unsigned)g.H) continue;
      for (int kw = 0; kw < g.k; ++kw) {
        const int w = ow * g.s - g.p + kw;
        if ((unsigned)w >= (unsigned)g.W) continue;
        float v[V];
        Vec<E>::load(x + ((n * g.H + h) * g.W + w) * g.C + cv * V, v);
        const int pos = kh * g.k + kw;
#pragma unroll
        for (int e = 0; e < V; ++e) {
          // first maximum wins; a NaN always takes over (torch's rule)
          if (!any || v[e] > m[e] || v[e] != v[e]) {
            m[e] = v[e];
            best[e] = pos;
          }
        }
        any = true;
      }
    }
    Vec<E>::store(y + i * V, m);
    uint32_t c0 = 0, c1 = 0;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      if (e < 4) c0 |= (uint32_t)best[e] << (8 * e);
      else c1 |= (uint32_t)best[e] << (8 * (e - 4));
    }
    if (V == 4) {
      *reinterpret_cast<uint32_t*>(code + i * V) = c0;
    } else {
      *reinterpret_cast<uint2*>(code + i * V) = make_uint2(c0, c1);
    }
  }
}

template <typename E>
__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const E* __restrict__ gy,
                                                          const uint8_t* __restrict__ code,
                                                          E* __restrict__ gx, int64_t total,
                                                          PoolGeom g) {
  constexpr int V = Vec<E>::N;
  const int CV = g.C / V;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    const int cv = (int)(i % CV);
    const int64_t pix = i / CV;
    const int w = (int)(pix % g.W);
    const int64_t q = pix / g.W;
    const int h = (int)(q % g.H);
    const int64_t n = q / g.H;
    float a[V];
#pragma unroll
    for (int e = 0; e < V; ++e) a[e] = 0.f;
    // windows oh with oh * s - p <= h <= oh * s - p + k - 1, ascending
    const int hp = h + g.p, wp = w + g.p;
    int oh0 = hp - g.k + 1 > 0 ? (hp - g.k + 1 + g.s - 1) / g.s : 0;
    int oh1 = hp / g.s;
    if (oh1 > g.OH - 1) oh1 = g.OH - 1;
    int ow0 = wp - g.k + 1 > 0 ? (wp - g.k + 1 + g.s - 1) / g.s : 0;
    int ow1 = wp / g.s;
    if (ow1 > g.OW - 1) ow1 = g.OW - 1;
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int kh = hp - oh * g.s;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int kw = wp - ow * g.s;
        const int pos = kh * g.k + kw;
        const int64_t o = ((n * g.OH + oh) * g.OW + ow) * g.C + cv * V;
        uint8_t cd[V];
        if (V == 4) {
          const uint32_t c = *reinterpret_cast<const uint32_t*>(code + o);
#pragma unroll
          for (int e = 0; e < V; ++e) cd[e] = (uint8_t)(c >> (8 * (e & 3)));
        } else {
          const uint2 c = *reinterpret_cast<const uint2*>(code + o);
#pragma unroll
          for (int e = 0; e < V; ++e)
            cd[e] = (uint8_t)((e < 4 ? c.x : c.y) >> (8 * (e & 3)));
        }
        bool hit = false;
#pragma unroll
        for (int e = 0; e < V; ++e) hit |= cd[e] == pos;
        if (!hit) continue;
        float v[V];
        Vec<E>::load(gy + o, v);
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (cd[e] == pos) a[e] += v[e];
      }
    }
    Vec<E>::store(gx + i * V, a);
  }
}

inline unsigned grid_for(int64_t n) {
  int64_t b = ceil_div(n, 256);
  if (b > 16384) b = 16384;
  return (unsigned)(b > 0 ? b : 1);
}

}  // namespace

// dtype: kF32 (C % 4 == 0) or kBF16 (C % 8 == 0); host checks shapes
void maxpool_nhwc_fwd(int dtype, const void* x, void* y, uint8_t* code, int N, int H, int W,
                      int C, int OH, int OW, int k, int s, int p, hipStream_t st) {
  const PoolGeom g{H, W, C, OH, OW, k, s, p};
  if (dtype == kBF16) {
    const int64_t total = (int64_t)N * OH * OW * (C / 8);
    if (total == 0) return;
    maxpool_fwd_kernel<uint16_t><<<grid_for(total), 256, 0, st>>>(
        (const uint16_t*)x, (uint16_t*)y, code, total, g);
  } else {
    const int64_t total = (int64_t)N * OH * OW * (C / 4);
    if (total == 0) return;
    maxpool_fwd_kernel<float><<<grid_for(total), 256, 0, st>>>((const float*)x, (float*)y, code,
                                                               total, g);
  }
}

void maxpool_nhwc_bwd(int dtype, const void* gy, const uint8_t* code, void* gx, int N, int H,
                      int W, int C, int OH, int OW, int k, int s, int p, hipStream_t st) {
  const PoolGeom g{H, W, C, OH, OW, k, s, p};
  if (dtype == kBF16) {
    const int64_t total = (int64_t)N * H * W * (C / 8);
    if (total == 0) return;
    maxpool_bwd_kernel<uint16_t><<<grid_for(total), 256, 0, st>>>(
        (const uint16_t*)gy, code, (uint16_t*)gx, total, g);
  } else {
    const int64_t total = (int64_t)N * H * W * (C / 4);
    if (total == 0) return;
    maxpool_bwd_kernel<float><<<grid_for(total), 256, 0, st>>>((const float*)gy, code,
                                                               (float*)gx, total, g);
  }
}

}  // namespace kfac
