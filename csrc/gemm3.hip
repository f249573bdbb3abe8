// K-HIP-4: grouped fp32 GEMM for the per-step K-FAC preconditioning, on
// bf16 MFMA with a three-term split ("bf16x3").
//
// Every step the eigen method computes, for every layer l (reference
// kfac/layers/eigen.py:349-384):
//     V1 = QG^T [Wg | bg] QA,   V2 = V1 (.) S,   P = QG V2 QA^T
// i.e. four dependent fp32 GEMMs per layer (S = 1/(dG (x) dA + damping) or
// the precomputed dGdA).  ResNet-50 has 54 layers with shapes from 64x64 to
// 512x4608 (K up to 4608): ~310 GFLOP/step.  The reference issues 4 cuBLAS
// calls + elementwise ops per layer; on MI355X that is ~220 launches per
// step, most of them too small to fill 256 CUs, and fp32 MFMA runs at
// 1/16 of the bf16 rate (v_mfma_f32_32x32x2_f32: 64 cyc/SIMD vs 32 cyc for
// a 32x32x16 bf16 MFMA of 8x the FLOPs).
//
// Here each chain step is ONE launch over all layers ("grouped GEMM"):
//   * a device descriptor table lists the layers (sorted heavy-K first so
//     the long tiles start first); a block finds its layer by binary search
//     over per-layer tile prefix sums;
//   * blockIdx -> tile mapping is XCD-aware: hardware dispatches block b to
//     XCD b % 8, so chunks of CH consecutive tiles (same A row panel) are
//     given to one XCD to share its L2, chunks round-robin across XCDs so
//     the heavy-first order is kept on every XCD;
//   * fp32 operands are split on the way into LDS: x = hi + lo with
//     hi = bf16_rn(x), lo = bf16_rn(x - hi), and A.B is accumulated in fp32
//     as hi.hi + hi.lo + lo.hi (3 bf16 MFMAs instead of 8 fp32 MFMAs per
//     32x32x16 block; dropped lo.lo and the representation error give a
//     relative error ~1e-5 per product -- fp32-class, far tighter than TF32);
//   * the A operand can carry one extra column from a vector (the bias
//     gradient of [Wg | bg], so the reference's torch.cat is never built);
//   * the epilogue applies the eigenvalue scaling S (matrix dGdA or vectors
//     dG, dA with damping) before the store, so V1 never round-trips.
//
// Tiling: 128x128 output tile per 256-thread block (4 waves in 2x2, 64x64
// each = 2x2 MFMA 32x32 accumulators), BK = 32, operands register-staged and
// split while being written to LDS; the LDS tile is double-buffered so the
// split + store of k-tile kt+1 overlaps the MFMAs of k-tile kt (the split's
// VALU work -- v_cvt_pk_bf16_f32 pairs -- is comparable to the MFMA time).  LDS layouts per operand:
//   k-contiguous in memory ([m][k]): LDS [m][40] bf16, fragment = one
//     ds_read_b128 (8 consecutive k) -- rows 80 B apart: conflict-free;
//   m-contiguous in memory ([k][m]): LDS [k][160] bf16, fragment = two
//     ds_read_b64_tr_b16 (transposing read).
#include "common.h"

#include <cstdlib>
#include <cstring>
#include "descs.h"

namespace kfac {


namespace {

constexpr int GT = 128;   // output tile edge
constexpr int GK = 32;    // k per LDS tile
constexpr int GNT = 256;  // threads per block
constexpr int LDK = 40;   // k-contig LDS row (32 + 8 pad) in shorts
constexpr int LDM = 160;  // m-contig LDS row (128 + 32 pad) in shorts
#ifndef GEMM3_CH
#define GEMM3_CH 4
#endif
#ifndef GEMM3_GM
#define GEMM3_GM 8
#endif
constexpr int CH = GEMM3_CH;  // consecutive tiles per XCD chunk
constexpr int GM = GEMM3_GM;  // tile rows per column group (L2 reuse)

// diagnostic builds only (tools/gemm3_bench.cpp): drop a phase to price it
#ifndef GEMM3_DIAG
#define GEMM3_DIAG 0  // 1: no global loads, 2: no LDS stores, 3: no MFMA
#endif

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf16 __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

__device__ __forceinline__ int find_tile_layer(const GemmDesc* d, int n, int t) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].tile_start <= t) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f2_t __attribute__((ext_vector_type(2)));

// x = hi + lo with hi = bf16_rn(x), lo = bf16_rn(x - hi): two
// v_cvt_pk_bf16_f32 (RNE) + mask/shift/sub per pair of values
__device__ __forceinline__ void split2(float x0, float x1, uint32_t& hi, uint32_t& lo) {
  const f2_t x = {x0, x1};
  hi = __builtin_bit_cast(uint32_t, __builtin_convertvector(x, bf16x2_t));
  const float h0 = __uint_as_float(hi << 16);
  const float h1 = __uint_as_float(hi & 0xFFFF0000u);
  const f2_t r = {x0 - h0, x1 - h1};
  lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf16x2_t));
}

__device__ __forceinline__ void split4(const float4 v, v4i16& hi, v4i16& lo) {
  uint32_t h0, l0, h1, l1;
  split2(v.x, v.y, h0, l0);
  split2(v.z, v.w, h1, l1);
  const uint2 hh = make_uint2(h0, h1), ll = make_uint2(l0, l1);
  hi = __builtin_bit_cast(v4i16, hh);
  lo = __builtin_bit_cast(v4i16, ll);
}

// one operand's staging registers: 4 float4 per thread per k-tile
struct Stage {
  float4 r[4];
  // bit p set: row group p is valid.  Loads land raw in r[] and the zeroing
  // of out-of-range rows waits until the split (stage_get): a select right
  // after the load made the compiler wait for the load there, before the
  // MFMAs of the current k-tile, and the prefetch never overlapped them.
  uint32_t ok;
};

__device__ __forceinline__ float4 stage_get(const Stage& st, int p) {
  return ((st.ok >> p) & 1u) ? st.r[p] : make_float4(0.f, 0.f, 0.f, 0.f);
}

// Pointers come out of the descriptor table, so the compiler cannot infer
// their address space and would emit FLAT loads (which also count on
// lgkmcnt and serialise against the LDS traffic): cast to global.
typedef const float __attribute__((address_space(1)))* gptr_t;
typedef float f4v_t __attribute__((ext_vector_type(4)));
typedef const f4v_t __attribute__((address_space(1)))* gptr4_t;

__device__ __forceinline__ float4 gload4(const float* p) {
  const f4v_t v = *(gptr4_t)(p);
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float gload(const float* p) {
  return *(gptr_t)(p);
}

// k-contiguous operand: rows [r0, r0+128) of a [rows][ld] matrix, columns
// [k0, k0+32).  Thread t: chunk = t & 7 (4 columns), row = (t >> 3) + 32p.
// Edge tiles load at clamped in-bounds addresses and zero afterwards: a
// load inside a per-row bounds branch made the compiler wait for each one
// before the next (194 `s_waitcnt vmcnt(0)` for 356 loads in the 1x1
// convolution kernel), so a partial tile -- every tile of a 64-wide
// operand -- ran one memory round trip per row.
__device__ __forceinline__ void load_kc(Stage& st, const float* __restrict__ P,
                                        const float* __restrict__ extra,
                                        int64_t ld, int rows, int r0,
                                        int kmain, int k0, bool vec) {
  const int t = threadIdx.x;
  const int c = k0 + (t & 7) * 4;
  if (vec && k0 + GK <= kmain) {
    // whole k-tile inside the matrix: float4 loads at clamped rows
    uint32_t ok = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int r = r0 + (t >> 3) + 32 * p;
      ok |= (r < rows ? 1u : 0u) << p;
      st.r[p] = gload4(P + (int64_t)(r < rows ? r : rows - 1) * ld + c);
    }
    st.ok = ok;
    return;
  }
  // k tail (or unaligned rows): scalar loads at clamped (row, k), the
  // optional extra column k == kmain from its own vector
  float tmp[4][4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = r0 + (t >> 3) + 32 * p;
    const int rc = r < rows ? r : rows - 1;
    const float* row = P + (int64_t)rc * ld;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = c + e;
      tmp[p][e] = gload(row + (k < kmain ? k : kmain - 1));
    }
  }
  float ex[4] = {0.f, 0.f, 0.f, 0.f};
  const bool has_extra = extra != nullptr && kmain >= c && kmain < c + 4;
  if (has_extra) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int r = r0 + (t >> 3) + 32 * p;
      ex[p] = gload(extra + (r < rows ? r : rows - 1));
    }
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const bool rok = r0 + (t >> 3) + 32 * p < rows;
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = c + e;
      o[e] = !rok ? 0.f : k < kmain ? tmp[p][e] : (has_extra && k == kmain) ? ex[p] : 0.f;
    }
    st.r[p] = make_float4(o[0], o[1], o[2], o[3]);
  }
  st.ok = 0xFu;
}

// The same loads for operands whose k-tiles are all whole and float4-able
// (K % 32 == 0, 16-byte rows: every convolution GEMM): no scalar tail path
// in the loop, whose register merge with the float4 path made the compiler
// wait for the prefetch before the current k-tile's MFMAs.
__device__ __forceinline__ void load_kc_v(Stage& st, const float* __restrict__ P, int64_t ld,
                                          int rows, int r0, int k0) {
  const int t = threadIdx.x;
  const int c = k0 + (t & 7) * 4;
  uint32_t ok = 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = r0 + (t >> 3) + 32 * p;
    ok |= (r < rows ? 1u : 0u) << p;
    st.r[p] = gload4(P + (int64_t)(r < rows ? r : rows - 1) * ld + c);
  }
  st.ok = ok;
}

__device__ __forceinline__ void load_mc_v(Stage& st, const float* __restrict__ P, int64_t ld,
                                          int cols, int m0, int K, int k0) {
  const int t = threadIdx.x;
  const int m = m0 + (t & 31) * 4;
  const bool cok = m < cols;
  const int mc = cok ? m : cols - 4;
  uint32_t ok = 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int k = k0 + (t >> 5) + 8 * p;
    ok |= (cok && k < K ? 1u : 0u) << p;
    st.r[p] = gload4(P + (int64_t)(k < K ? k : K - 1) * ld + mc);
  }
  st.ok = ok;
}

__device__ __forceinline__ void store_kc(const Stage& st, short* Lh, short* Ll) {
  const int t = threadIdx.x;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = (t >> 3) + 32 * p;
    v4i16 h, l;
    split4(stage_get(st, p), h, l);
    *reinterpret_cast<v4i16*>(Lh + r * LDK + (t & 7) * 4) = h;
    *reinterpret_cast<v4i16*>(Ll + r * LDK + (t & 7) * 4) = l;
  }
}

// m-contiguous operand: k-rows [k0, k0+32) of a [K][ld] matrix, columns
// [m0, m0+128).  Thread t: chunk = t & 31 (4 columns), krow = (t >> 5) + 8p.
// Clamped loads, masked afterwards (see load_kc).
__device__ __forceinline__ void load_mc(Stage& st, const float* __restrict__ P,
                                        int64_t ld, int cols, int m0, int K,
                                        int k0, bool vec) {
  const int t = threadIdx.x;
  const int m = m0 + (t & 31) * 4;
  if (vec && (cols & 3) == 0) {
    // columns come in whole float4 groups: a group is in or out
    const bool cok = m < cols;
    const int mc = cok ? m : cols - 4;
    uint32_t ok = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int k = k0 + (t >> 5) + 8 * p;
      ok |= (cok && k < K ? 1u : 0u) << p;
      st.r[p] = gload4(P + (int64_t)(k < K ? k : K - 1) * ld + mc);
    }
    st.ok = ok;
    return;
  }
  float tmp[4][4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int k = k0 + (t >> 5) + 8 * p;
    const float* row = P + (int64_t)(k < K ? k : K - 1) * ld;
#pragma unroll
    for (int e = 0; e < 4; ++e) tmp[p][e] = gload(row + (m + e < cols ? m + e : cols - 1));
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const bool kok = k0 + (t >> 5) + 8 * p < K;
    st.r[p] = make_float4(kok && m < cols ? tmp[p][0] : 0.f, kok && m + 1 < cols ? tmp[p][1] : 0.f,
                          kok && m + 2 < cols ? tmp[p][2] : 0.f,
                          kok && m + 3 < cols ? tmp[p][3] : 0.f);
  }
  st.ok = 0xFu;
}

__device__ __forceinline__ void store_mc(const Stage& st, short* Lh, short* Ll) {
  const int t = threadIdx.x;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int k = (t >> 5) + 8 * p;
    v4i16 h, l;
    split4(stage_get(st, p), h, l);
    *reinterpret_cast<v4i16*>(Lh + k * LDM + (t & 31) * 4) = h;
    *reinterpret_cast<v4i16*>(Ll + k * LDM + (t & 31) * 4) = l;
  }
}

// ---- pre-split operands: bf16 hi/lo interleaved per 4 consecutive
// elements ([h0 h1 h2 h3 l0 l1 l2 l3] = 16 B, the footprint of 4 fp32), so
// a group is read with the fp32 operand's float4 offsets and lands in a
// Stage float4 as {hi01, hi23, lo01, lo23}.  Rows / k extents are multiples
// of 4 (checked on the host), so groups never straddle an edge.
__device__ __forceinline__ void load_kc_hl(Stage& st, const float* __restrict__ P, int64_t ld,
                                           int rows, int r0, int kmain, int k0) {
  const int t = threadIdx.x;
  const int c = k0 + (t & 7) * 4;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = r0 + (t >> 3) + 32 * p;
    st.r[p] = (r < rows && c < kmain) ? gload4(P + (int64_t)r * ld + c)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  st.ok = 0xFu;
}

__device__ __forceinline__ void load_mc_hl(Stage& st, const float* __restrict__ P, int64_t ld,
                                           int cols, int m0, int K, int k0) {
  const int t = threadIdx.x;
  const int m = m0 + (t & 31) * 4;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int k = k0 + (t >> 5) + 8 * p;
    st.r[p] = (k < K && m < cols) ? gload4(P + (int64_t)k * ld + m)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  st.ok = 0xFu;
}

__device__ __forceinline__ void unpack_hl(const float4 v, v4i16& hi, v4i16& lo) {
  hi = __builtin_bit_cast(v4i16, make_uint2(__float_as_uint(v.x), __float_as_uint(v.y)));
  lo = __builtin_bit_cast(v4i16, make_uint2(__float_as_uint(v.z), __float_as_uint(v.w)));
}

__device__ __forceinline__ void store_kc_hl(const Stage& st, short* Lh, short* Ll) {
  const int t = threadIdx.x;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = (t >> 3) + 32 * p;
    v4i16 h, l;
    unpack_hl(st.r[p], h, l);
    *reinterpret_cast<v4i16*>(Lh + r * LDK + (t & 7) * 4) = h;
    *reinterpret_cast<v4i16*>(Ll + r * LDK + (t & 7) * 4) = l;
  }
}

__device__ __forceinline__ void store_mc_hl(const Stage& st, short* Lh, short* Ll) {
  const int t = threadIdx.x;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int k = (t >> 5) + 8 * p;
    v4i16 h, l;
    unpack_hl(st.r[p], h, l);
    *reinterpret_cast<v4i16*>(Lh + k * LDM + (t & 31) * 4) = h;
    *reinterpret_cast<v4i16*>(Ll + k * LDM + (t & 31) * 4) = l;
  }
}

// ---- implicit im2col (the fp32 3x3 convolutions, ops/conv.py): A is the
// NHWC input x[N][H][W][C] read as the [N*Ho*Wo][kh*kw*C] patch matrix,
// k = (tap i*kw + j) * C + c -- the order of a channels_last weight
// [Cout][kh][kw][C], so B is the weight as stored.  C % 32 == 0 (host
// check): a 32-wide k-tile lies inside one tap, each thread's 4 channels
// are one float4.  Rows are decoded once per tile (conv_rows); every load is
// issued at a clamped in-bounds address and zeroed afterwards (padding and
// rows past M), so a thread's four row loads stay in flight together.
struct PatchGeom {
  int32_t H, W, C, Ho, Wo, kw, stride, pad, kh;
};

struct ConvRows {
  int pix[4];  // n * H * W of the row's image
  int hb[4];   // ho * stride - pad (very negative past M: always padding)
  int wb[4];   // wo * stride - pad
};

__device__ __forceinline__ void conv_rows(ConvRows& cr, const PatchGeom& g, int M, int r0) {
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = r0 + (threadIdx.x >> 3) + 32 * p;
    const bool ok = r < M;
    const int rr = ok ? r : 0;
    const int wo = rr % g.Wo;
    const int q = rr / g.Wo;
    const int ho = q % g.Ho;
    const int n = q / g.Ho;
    cr.pix[p] = n * g.H * g.W;
    cr.hb[p] = ok ? ho * g.stride - g.pad : -(1 << 28);
    cr.wb[p] = wo * g.stride - g.pad;
  }
}

// (C % 4 == 0 in general: a thread's 4 channels lie in one tap; with C %
// 32 != 0 -- the 4-channel padded stem -- a k-tile spans several taps and
// k may run past K in the last tile)
__device__ __forceinline__ void load_kc_conv(Stage& st, const float* __restrict__ X,
                                             const PatchGeom& g, const ConvRows& cr, int k0,
                                             int K) {
  const int kk = k0 + (threadIdx.x & 7) * 4;
  const int tap = kk / g.C;
  const int c = kk - tap * g.C;
  const int i = tap / g.kw, j = tap - i * g.kw;
  const bool kok = kk < K;
  uint32_t ok = 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int hi = cr.hb[p] + i, wi = cr.wb[p] + j;
    const bool in = kok && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
    ok |= (in ? 1u : 0u) << p;
    st.r[p] = gload4(X + (in ? ((int64_t)(cr.pix[p] + hi * g.W + wi)) * g.C + c : 0));
  }
  st.ok = ok;
}

// B of the stride-1 input gradient: the flipped, transposed kernel read in
// place from the channels_last weight w[Co][kh][kw][Ci] (no flipped copy):
// B[k = (i, j, co)][n = ci] = w[co][kh-1-i][kw-1-j][ci], n-contiguous rows.
// The patches' C is Co, so a 32-row k-tile lies inside one tap.
__device__ __forceinline__ void load_mc_flipw(Stage& st, const float* __restrict__ Wt,
                                              const PatchGeom& g, int ncols, int n0, int k0) {
  const int t = threadIdx.x;
  const int n = n0 + (t & 31) * 4;
  const int tap = k0 / g.C;
  const int i = tap / g.kw, j = tap - i * g.kw;
  const int co0 = k0 - tap * g.C + (t >> 5);
  const int64_t tapoff = (int64_t)((g.kh - 1 - i) * g.kw + (g.kw - 1 - j)) * ncols;
  const bool ok = n < ncols;  // ncols % 4 == 0 (host check)
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int co = co0 + 8 * p;
    const int64_t off = ok ? (int64_t)co * g.kh * g.kw * ncols + tapoff + n : 0;
    st.r[p] = gload4(Wt + off);
  }
  st.ok = ok ? 0xFu : 0u;
}

// B of a weight gradient: the patch matrix as [K = N*Ho*Wo pixels][n =
// (tap, c)] rows (n-contiguous), gathered from the NHWC input.  Each k-row
// is decoded to (image, ho, wo) by a float reciprocal with an exact integer
// fix-up (pixel counts < 2^22); c % 4 == 0, so a thread's 4 columns share
// one tap.
__device__ __forceinline__ int fdivmod(int a, int b, float inv, int& r) {
  int q = __float2int_rz((float)a * inv);
  r = a - q * b;
  if (r < 0) { --q; r += b; }
  else if (r >= b) { ++q; r -= b; }
  return q;
}

__device__ __forceinline__ void load_mc_patch(Stage& st, const float* __restrict__ X,
                                              const PatchGeom& g, int ncols, int n0, int K,
                                              int k0) {
  const int t = threadIdx.x;
  const int n = n0 + (t & 31) * 4;
  const bool cok = n < ncols;
  const int nn = cok ? n : 0;
  const int tap = nn / g.C;
  const int c = nn - tap * g.C;
  const int i = tap / g.kw, j = tap - i * g.kw;
  const float inv_wo = 1.f / (float)g.Wo, inv_ho = 1.f / (float)g.Ho;
  uint32_t ok = 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int k = k0 + (t >> 5) + 8 * p;
    const int kc = k < K ? k : K - 1;
    int wo, ho;
    const int q = fdivmod(kc, g.Wo, inv_wo, wo);
    const int img = fdivmod(q, g.Ho, inv_ho, ho);
    const int hi = ho * g.stride - g.pad + i, wi = wo * g.stride - g.pad + j;
    const bool in = cok && k < K && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
    ok |= (in ? 1u : 0u) << p;
    st.r[p] = gload4(X + (in ? ((int64_t)((img * g.H + hi) * g.W + wi)) * g.C + c : 0));
  }
  st.ok = ok;
}

// fragment: lane l gets X[row = base + (l & 31)][k = kk + 8 (l >> 5) + 0..7]
__device__ __forceinline__ v8bf16 frag_kc(const short* L, int base, int kk) {
  const int l = threadIdx.x & 63;
  const v8i16 v = *reinterpret_cast<const v8i16*>(L + (base + (l & 31)) * LDK + kk + 8 * (l >> 5));
  return __builtin_bit_cast(v8bf16, v);
}

// fragment from a [k][m] LDS tile: lane l gets X[k = kk + 8h + j][m = base + (l & 31)]
__device__ __forceinline__ v8bf16 frag_mc(const short* L, int base, int kk) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4;
  const int i = l & 15;
  const int q = i >> 2, p = i & 3;
  const int col = base + 16 * (g & 1) + 4 * p;
  const int krow = kk + 8 * (g >> 1) + q;
  const short* a0 = L + krow * LDM + col;
  const short* a1 = a0 + 4 * LDM;
  v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)a0);
  v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)a1);
  v8i16 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(v8bf16, c);
}

// XCD-aware chunked remap of the block index (see header)
__device__ __forceinline__ int gemm3_tile_of_block() {
  const int b = blockIdx.x;
  const int xcd = b & 7, r = b >> 3;
  return ((r / CH) * 8 + xcd) * CH + (r % CH);
}

// one 128 x 128 output tile t of the GEMM described by d
// k-tiles [kt_begin, kt_begin + kt_count) of the reduction (split-K
// callers; kt_count < 0: to the end)
template <bool A_KC, bool B_KC, bool CONV = false, bool FLIPW = false, bool FASTLD = false,
          bool PATCHB = false, bool NARROW = false>
__device__ __forceinline__ void gemm3_tile(const GemmDesc& d, int t, const PatchGeom& g = {},
                                           int kt_begin = 0, int kt_count = -1) {
  constexpr int A_SZ = A_KC ? GT * LDK : GK * LDM;
  constexpr int B_SZ = B_KC ? GT * LDK : GK * LDM;
  constexpr int BUF = 2 * A_SZ + 2 * B_SZ;
  // double-buffered: the split + LDS store of k-tile kt+1 overlaps the
  // MFMAs on k-tile kt; one barrier per k-tile
  __shared__ __attribute__((aligned(16))) short lds[2 * BUF];

  // grouped order inside a layer: GM tile rows x one tile column, column
  // after column, so a chunk of CH consecutive tiles covers a GM x CH/GM
  // block of C whose A and B panels are shared in the XCD's L2
  const int tl = t - d.tile_start;
  const int tiles_m = (d.M + GT - 1) / GT;
  const int per_group = GM * d.tiles_n;
  const int first_m = (tl / per_group) * GM;
  const int gm = min(tiles_m - first_m, GM);
  const int in_group = tl % per_group;
  const int m0 = (first_m + in_group % gm) * GT;
  const int n0 = (in_group / gm) * GT;
  const bool avec = d.vec & 1, bvec = (d.vec >> 1) & 1;
  const bool a_hl = d.Ah != nullptr, b_hl = d.Bh != nullptr;

  const int w = threadIdx.x >> 6;
  const int l = threadIdx.x & 63;
  const int wr = w >> 1, wc = w & 1;
  // NARROW (a launch whose N <= 64: a 64-channel convolution output): the
  // four waves split the 128 rows 32 each over all 64 columns instead of
  // two of them multiplying zero columns.  Wave w owns rows rb + 32 i
  // (i < ni) and columns cb + 32 j.  A template parameter, so the wide
  // tiles' index arithmetic stays compile-time.
  constexpr bool narrow = NARROW;
  const int rb = narrow ? w * 32 : wr * 64;
  const int cb = narrow ? 0 : wc * 64;
  constexpr int ni = narrow ? 1 : 2;

  v16f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // two register stages: the global loads of k-tile kt+2 are issued while
  // k-tile kt is multiplied, so each load has two k-tiles of MFMA time
  // (plus the co-resident block's) to land before it is split and stored
  Stage sa0, sb0, sa1, sb1;
  ConvRows cr;
  if constexpr (CONV) conv_rows(cr, g, d.M, m0);
  auto load = [&](Stage& sa, Stage& sb, int k0) {
    if constexpr (GEMM3_DIAG == 1) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        sa.r[p] = make_float4(k0, 1.f, 2.f, 3.f);
        sb.r[p] = make_float4(k0, 1.f, 2.f, 3.f);
      }
      sa.ok = sb.ok = 0xFu;
      return;
    }
    if constexpr (CONV) {
      load_kc_conv(sa, d.A, g, cr, k0, d.K);
    } else if constexpr (FASTLD && A_KC) {
      load_kc_v(sa, d.A, d.lda, d.M, m0, k0);
    } else if constexpr (FASTLD) {
      load_mc_v(sa, d.A, d.lda, d.M, m0, d.K, k0);
    } else if constexpr (A_KC) {
      if (a_hl) load_kc_hl(sa, (const float*)d.Ah, d.lda, d.M, m0, d.Kmain, k0);
      else load_kc(sa, d.A, d.A_extra, d.lda, d.M, m0, d.Kmain, k0, avec);
    } else {
      if (a_hl) load_mc_hl(sa, (const float*)d.Ah, d.lda, d.M, m0, d.K, k0);
      else load_mc(sa, d.A, d.lda, d.M, m0, d.K, k0, avec);
    }
    if constexpr (PATCHB) {
      load_mc_patch(sb, d.B, g, d.N, n0, d.K, k0);
    } else if constexpr (FLIPW) {
      load_mc_flipw(sb, d.B, g, d.N, n0, k0);
    } else if constexpr (FASTLD && B_KC) {
      load_kc_v(sb, d.B, d.ldb, d.N, n0, k0);
    } else if constexpr (FASTLD) {
      load_mc_v(sb, d.B, d.ldb, d.N, n0, d.K, k0);
    } else if constexpr (B_KC) {
      if (b_hl) load_kc_hl(sb, (const float*)d.Bh, d.ldb, d.N, n0, d.K, k0);
      else load_kc(sb, d.B, nullptr, d.ldb, d.N, n0, d.K, k0, bvec);
    } else {
      if (b_hl) load_mc_hl(sb, (const float*)d.Bh, d.ldb, d.N, n0, d.K, k0);
      else load_mc(sb, d.B, d.ldb, d.N, n0, d.K, k0, bvec);
    }
  };
  auto store = [&](const Stage& sa, const Stage& sb, short* buf) {
    if constexpr (GEMM3_DIAG == 2) {
      if (sa.r[0].x == 12345.f && sb.r[3].w == 54321.f) buf[threadIdx.x] = 1;
      return;
    }
    if constexpr (A_KC) {
      if (a_hl) store_kc_hl(sa, buf, buf + A_SZ);
      else store_kc(sa, buf, buf + A_SZ);
    } else {
      if (a_hl) store_mc_hl(sa, buf, buf + A_SZ);
      else store_mc(sa, buf, buf + A_SZ);
    }
    if constexpr (B_KC) {
      if (b_hl) store_kc_hl(sb, buf + 2 * A_SZ, buf + 2 * A_SZ + B_SZ);
      else store_kc(sb, buf + 2 * A_SZ, buf + 2 * A_SZ + B_SZ);
    } else {
      if (b_hl) store_mc_hl(sb, buf + 2 * A_SZ, buf + 2 * A_SZ + B_SZ);
      else store_mc(sb, buf + 2 * A_SZ, buf + 2 * A_SZ + B_SZ);
    }
  };
  auto compute = [&](const short* cur) {
    const short* Ah = cur;
    const short* Al = cur + A_SZ;
    const short* Bh = cur + 2 * A_SZ;
    const short* Bl = cur + 2 * A_SZ + B_SZ;
#pragma unroll
    for (int kk = 0; kk < GK; kk += 16) {
      v8bf16 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int am = rb + (i < ni ? i : 0) * 32;
        const int bn = cb + i * 32;
        if (i < ni) {
          if constexpr (A_KC) {
            ah[i] = frag_kc(Ah, am, kk);
            al[i] = frag_kc(Al, am, kk);
          } else {
            ah[i] = frag_mc(Ah, am, kk);
            al[i] = frag_mc(Al, am, kk);
          }
        }
        if constexpr (B_KC) {
          bh[i] = frag_kc(Bh, bn, kk);
          bl[i] = frag_kc(Bl, bn, kk);
        } else {
          bh[i] = frag_mc(Bh, bn, kk);
          bl[i] = frag_mc(Bl, bn, kk);
        }
      }
      if constexpr (GEMM3_DIAG == 3) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[i][i][0] += (float)(ah[i][0] + al[i][1] + bh[i][2] + bl[i][3]);
        continue;
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (i >= ni) continue;  // uniform: narrow tiles have one row block
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
      }
    }
  };
  // iteration kt: LDS buf[kt&1] holds tile kt, stage (kt+1)&1 holds tile
  // kt+1 (in flight), stage kt&1 is free for tile kt+2
  const int kb = kt_begin * GK;
  auto step = [&](int kt, int nt, Stage& fa, Stage& fb, Stage& na, Stage& nb) {
    if (kt + 2 < nt) load(fa, fb, kb + (kt + 2) * GK);
    compute(lds + (kt & 1) * BUF);
    if (kt + 1 < nt) store(na, nb, lds + ((kt + 1) & 1) * BUF);
    __syncthreads();
  };

  const int kt_all = (d.K + GK - 1) / GK - kt_begin;
  const int ntiles = kt_count < 0 ? kt_all : min(kt_count, kt_all);
  load(sa0, sb0, kb);
  if (ntiles > 1) load(sa1, sb1, kb + GK);
  store(sa0, sb0, lds);
  __syncthreads();
  for (int kt = 0; kt < ntiles; kt += 2) {
    step(kt, ntiles, sa0, sb0, sa1, sb1);
    if (kt + 1 < ntiles) step(kt + 1, ntiles, sa1, sb1, sa0, sb0);
  }

  // epilogue: C/D layout col = lane & 31, row = (reg&3) + 8 (reg>>2) + 4 (lane>>5)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (i >= ni) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + cb + j * 32 + (l & 31);
      if (n >= d.N) continue;
      const float dan = d.da != nullptr ? gload(d.da + n) : 0.f;
      // the addend's 16 values loaded together at clamped rows (one memory
      // round trip, not one per element)
      float dv[16];
      if (d.D != nullptr) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + rb + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
          dv[e] = gload(d.D + (int64_t)(m < d.M ? m : d.M - 1) * d.ldc + n);
        }
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + rb + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
        if (m >= d.M) continue;
        float v = acc[i][j][e];
        if (d.D != nullptr) v += dv[e];
        if (d.S != nullptr) v *= gload(d.S + (int64_t)m * d.lds + n);
        else if (d.dg != nullptr) v = v / (gload(d.dg + m) * dan + d.damping);
        *(float __attribute__((address_space(1)))*)(d.C + (int64_t)m * d.ldc + n) = v;
      }
    }
  }
  if (d.bnpart != nullptr) {
    // BN statistics per 64-row half tile: lanes l and l + 32 hold the two
    // interleaved row sets of a column; rows past M are zero.  A narrow
    // tile's waves own 32 rows each: waves 2h and 2h + 1 are summed in LDS
    // (free after the main loop's last barrier) into half h.
    typedef float __attribute__((address_space(1)))* gout_t;
    float sj[2], qj[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (i >= ni) continue;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + rb + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
          const float v = m < d.M ? acc[i][j][e] : 0.f;
          s += v;
          q += v * v;
        }
      }
      sj[j] = s + __shfl_xor(s, 32);
      qj[j] = q + __shfl_xor(q, 32);
    }
    int half = wr;
    bool writer = true;
    if constexpr (narrow) {
      float* red = reinterpret_cast<float*>(lds);  // [4 waves][2 j][2][32]
      if (l < 32) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          red[((w * 2 + j) * 2 + 0) * 32 + l] = sj[j];
          red[((w * 2 + j) * 2 + 1) * 32 + l] = qj[j];
        }
      }
      __syncthreads();
      half = w >> 1;
      writer = (w & 1) == 0;
      if (writer && l < 32) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          sj[j] += red[(((w + 1) * 2 + j) * 2 + 0) * 32 + l];
          qj[j] += red[(((w + 1) * 2 + j) * 2 + 1) * 32 + l];
        }
      }
    }
    const int prow = (m0 / GT) * 2 + half;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + cb + j * 32 + (l & 31);
      if (writer && l < 32 && n < d.N) {
        ((gout_t)d.bnpart)[(int64_t)(prow * 2) * d.N + n] = sj[j];
        ((gout_t)d.bnpart)[(int64_t)(prow * 2 + 1) * d.N + n] = qj[j];
      }
    }
  }
}

template <bool A_KC, bool B_KC>
__global__ void __launch_bounds__(GNT, 2)
gemm3_kernel(const GemmDesc* __restrict__ descs, int nlayers, int total_tiles) {
  const int t = gemm3_tile_of_block();
  if (t >= total_tiles) return;
  const GemmDesc d = descs[find_tile_layer(descs, nlayers, t)];
  gemm3_tile<A_KC, B_KC>(d, t);
}

// one GEMM whose descriptor travels in the kernel arguments: no device
// table to upload, so a launch is one graph-capturable kernel node (the
// fp32 1x1 convolutions, ops/conv.py)
// split-K as gemm3_conv_kernel: block b covers tile b % tiles of split
// b / tiles, whose partial goes to C + split * split_stride
template <bool A_KC, bool B_KC, bool FASTLD, bool NARROW>
__global__ void __launch_bounds__(GNT, 2)
gemm3_single_kernel(const GemmDesc d, int tiles, int splits, int kt_per, int64_t split_stride) {
  const int b = gemm3_tile_of_block();
  if (b >= tiles * splits) return;
  if (splits == 1) {
    gemm3_tile<A_KC, B_KC, false, false, FASTLD, false, NARROW>(d, b);
    return;
  }
  const int z = b / tiles;
  GemmDesc dz = d;
  dz.C = d.C + (int64_t)z * split_stride;
  gemm3_tile<A_KC, B_KC, false, false, FASTLD, false, NARROW>(dz, b - z * tiles, {},
                                                             z * kt_per, kt_per);
}

// implicit-GEMM convolution: C[N*Ho*Wo][Cout] = patches(x) . w^T, the
// descriptor and the geometry by value
// split-K: block b covers tile (b' % tiles) of split (b' / tiles) and
// writes its partial sum to C + split * split_stride (the host sums them)
template <bool FLIPW, bool FASTB, bool NARROW>
__global__ void __launch_bounds__(GNT, 2)
gemm3_conv_kernel(const GemmDesc d, const PatchGeom g, int tiles, int splits, int kt_per,
                  int64_t split_stride) {
  const int b = gemm3_tile_of_block();
  if (b >= tiles * splits) return;
  const int z = b / tiles;
  GemmDesc dz = d;
  dz.C = d.C + (int64_t)z * split_stride;
  gemm3_tile<true, !FLIPW, true, FLIPW, FASTB, false, NARROW>(dz, b - z * tiles, g, z * kt_per,
                                                             kt_per);
}

// weight gradient of the implicit-GEMM convolution: dW[Co][(tap, c)] =
// dy^T . patches(x), split-K over the pixels
__global__ void __launch_bounds__(GNT, 2)
gemm3_wgrad_kernel(const GemmDesc d, const PatchGeom g, int tiles, int splits, int kt_per,
                   int64_t split_stride) {
  const int b = gemm3_tile_of_block();
  if (b >= tiles * splits) return;
  const int z = b / tiles;
  GemmDesc dz = d;
  dz.C = d.C + (int64_t)z * split_stride;
  gemm3_tile<false, false, false, false, true, true>(dz, b - z * tiles, g, z * kt_per, kt_per);
}

}  // namespace

int gemm3_tile_edge() { return GT; }

int gemm3_grid(int total_tiles) {
  const int per = 8 * CH;
  return ((total_tiles + per - 1) / per) * per;
}

void gemm3_grouped(const GemmDesc* table, int nlayers, int total_tiles,
                   bool a_kc, bool b_kc, hipStream_t s) {
  if (nlayers <= 0 || total_tiles <= 0) return;
  const dim3 grid((unsigned)gemm3_grid(total_tiles));
  if (a_kc && b_kc) gemm3_kernel<true, true><<<grid, dim3(GNT), 0, s>>>(table, nlayers, total_tiles);
  else if (a_kc) gemm3_kernel<true, false><<<grid, dim3(GNT), 0, s>>>(table, nlayers, total_tiles);
  else if (b_kc) gemm3_kernel<false, true><<<grid, dim3(GNT), 0, s>>>(table, nlayers, total_tiles);
  else gemm3_kernel<false, false><<<grid, dim3(GNT), 0, s>>>(table, nlayers, total_tiles);
}

// splits > 1: d.C holds `splits` partial [M][ldc] outputs, split_stride
// elements apart, each over an equal share of whole k-tiles (every split
// non-empty: the host passes splits <= the k-tile count)
// the narrow-tile instantiation for launches with N <= 64
// (KFAC_GEMM3_NARROW=0: the square wave layout, for A/B runs)
static bool narrow_for(int N) {
  static const bool on = [] {
    const char* e = std::getenv("KFAC_GEMM3_NARROW");
    return e == nullptr || std::strcmp(e, "0") != 0;
  }();
  return on && N <= 64;
}

void gemm3_single(const GemmDesc& d, bool a_kc, bool b_kc, int splits, int64_t split_stride,
                  hipStream_t s) {
  const int tiles = ((d.M + GT - 1) / GT) * d.tiles_n;
  if (tiles <= 0 || d.K <= 0) return;
  const int kts = (d.K + GK - 1) / GK;
  if (splits < 1) splits = 1;
  if (splits > kts) splits = kts;
  const int per = (kts + splits - 1) / splits;
  splits = (kts + per - 1) / per;
  const dim3 grid((unsigned)gemm3_grid(tiles * splits));
  // whole float4-able k-tiles and 4-aligned m-contiguous extents: the
  // tail-free loaders
  const bool fast = d.K % GK == 0 && d.vec == 3 && d.A_extra == nullptr &&
                    (a_kc || d.M % 4 == 0) && (b_kc || d.N % 4 == 0);
  const bool nar = narrow_for(d.N);
#define G3S_(A, B, NW)                                                                        \
  (fast ? gemm3_single_kernel<A, B, true, NW><<<grid, dim3(GNT), 0, s>>>(d, tiles, splits, per, \
                                                                           split_stride)      \
        : gemm3_single_kernel<A, B, false, NW><<<grid, dim3(GNT), 0, s>>>(d, tiles, splits,    \
                                                                            per, split_stride))
#define G3S(A, B) (nar ? G3S_(A, B, true) : G3S_(A, B, false))
  if (a_kc && b_kc) G3S(true, true);
  else if (a_kc) G3S(true, false);
  else if (b_kc) G3S(false, true);
  else G3S(false, false);
#undef G3S
#undef G3S_
}

int gemm3_conv_splits(int N, int H, int W, int C, int Cout, int kh, int kw, int stride, int pad) {
  const int Ho = (H + 2 * pad - kh) / stride + 1;
  const int Wo = (W + 2 * pad - kw) / stride + 1;
  const int tiles = ((N * Ho * Wo + GT - 1) / GT) * ((Cout + GT - 1) / GT);
  const int kts = (kh * kw * C + GK - 1) / GK;
  // fill the chip (KFAC_CONV_SPLIT_TARGET blocks, default 256: one per CU),
  // keeping >= 8 k-tiles per split
  static const int target = [] {
    const char* e = std::getenv("KFAC_CONV_SPLIT_TARGET");
    const int v = e != nullptr ? std::atoi(e) : 256;
    return v > 0 ? v : 256;
  }();
  int sp = (target + tiles - 1) / tiles;
  if (sp > kts / 8) sp = kts / 8;
  if (sp < 1) sp = 1;
  // equal k-tile counts: every split non-empty
  const int per = (kts + sp - 1) / sp;
  return (kts + per - 1) / per;
}

// y: [splits][N*Ho*Wo][Cout] partials when splits > 1.  flipw: w is the
// forward weight [Cout_fwd = C][kh][kw][Cout] of a stride-1 convolution and
// the kernel applied is its flipped transpose (the input gradient of x is
// gemm3_conv(dy, w, flipw) with pad kh - 1 - pad)
void gemm3_conv(const float* x, const float* w, float* y, int N, int H, int W, int C, int Cout,
                int kh, int kw, int stride, int pad, int splits, bool flipw, hipStream_t s,
                float* bnpart) {
  const int Ho = (H + 2 * pad - kh) / stride + 1;
  const int Wo = (W + 2 * pad - kw) / stride + 1;
  GemmDesc d{};
  d.A = x;
  d.B = w;
  d.C = y;
  d.lda = C;
  d.ldb = (int64_t)kh * kw * C;
  d.ldc = Cout;
  d.M = N * Ho * Wo;
  d.N = Cout;
  d.K = kh * kw * C;
  d.Kmain = d.K;
  d.tiles_n = (Cout + GT - 1) / GT;
  d.vec = 3;
  d.bnpart = splits == 1 ? bnpart : nullptr;  // partial sums are not outputs
  const PatchGeom g{H, W, C, Ho, Wo, kw, stride, pad, kh};
  const int tiles = ((d.M + GT - 1) / GT) * d.tiles_n;
  if (tiles <= 0) return;
  const int kts = (d.K + GK - 1) / GK;
  const int per = (kts + splits - 1) / splits;
  const dim3 grid((unsigned)gemm3_grid(tiles * splits));
  const int64_t st = (int64_t)d.M * Cout;
#define G3C(FW, FB)                                                                         \
  (narrow_for(Cout)                                                                         \
       ? gemm3_conv_kernel<FW, FB, true><<<grid, dim3(GNT), 0, s>>>(d, g, tiles, splits, per, st) \
       : gemm3_conv_kernel<FW, FB, false><<<grid, dim3(GNT), 0, s>>>(d, g, tiles, splits, per, st))
  if (flipw) {  // host: C % 32 == 0 (whole taps per k-tile)
    d.ldb = Cout;
    G3C(true, true);
  } else if (d.K % GK == 0) {
    G3C(false, true);
  } else {
    G3C(false, false);
  }
#undef G3C
}

int gemm3_wgrad_splits(int pixels, int Cout, int kcols) {
  const int tiles = ((Cout + GT - 1) / GT) * ((kcols + GT - 1) / GT);
  const int kts = (pixels + GK - 1) / GK;
  // KFAC_WGRAD_SPLIT_BLOCKS (default 512): blocks the split-K aims for --
  // more splits fill the chip, fewer shrink the partial-sum pass
  static const int target = [] {
    const char* e = std::getenv("KFAC_WGRAD_SPLIT_BLOCKS");
    const int v = e != nullptr ? std::atoi(e) : 0;
    return v > 0 ? v : 512;
  }();
  int sp = (target + tiles - 1) / tiles;
  if (sp > kts / 8) sp = kts / 8;
  if (sp < 1) sp = 1;
  const int per = (kts + sp - 1) / sp;
  return (kts + per - 1) / per;
}

// dw: [splits][Cout][kh*kw*C] partials (splits from gemm3_wgrad_splits)
void gemm3_conv_wgrad(const float* x, const float* dy, float* dw, int N, int H, int W, int C,
                      int Cout, int kh, int kw, int stride, int pad, int splits, hipStream_t s) {
  const int Ho = (H + 2 * pad - kh) / stride + 1;
  const int Wo = (W + 2 * pad - kw) / stride + 1;
  GemmDesc d{};
  d.A = dy;
  d.B = x;
  d.C = dw;
  d.lda = Cout;
  d.ldb = 0;
  d.ldc = (int64_t)kh * kw * C;
  d.M = Cout;
  d.N = kh * kw * C;
  d.K = N * Ho * Wo;
  d.Kmain = d.K;
  d.tiles_n = (d.N + GT - 1) / GT;
  d.vec = 3;
    const PatchGeom g{H, W, C, Ho, Wo, kw, stride, pad, kh};
  const int tiles = ((d.M + GT - 1) / GT) * d.tiles_n;
  const int kts = (d.K + GK - 1) / GK;
  const int per = (kts + splits - 1) / splits;
  gemm3_wgrad_kernel<<<dim3((unsigned)gemm3_grid(tiles * splits)), dim3(GNT), 0, s>>>(
      d, g, tiles, splits, per, (int64_t)d.M * d.N);
}

}  // namespace kfac
