// K-HIP-1: Kronecker-factor SYRK on MFMA.
//
//   C[D,D] = beta * C + alpha * Xt^T Xt,   Xt = [X | 1] (bias) or X,
//   X: [N, K] row-major (row stride ldx), bf16 or fp32; C fp32.
//
// Replaces the reference's get_cov / append_bias_ones / EMA chain
// (kfac/layers/utils.py:7-58, kfac/layers/base.py:344-404):
//   * the bias "ones" column is synthesised by the tile loader (no cat),
//   * the 1/N and conv 1/spatial^2 scalings and the EMA weights fold into
//     alpha/beta (C = decay*C + (1-decay)*scale*X^T X in ONE pass),
//   * only upper-triangle tiles are computed; the lower triangle is written
//     as the mirror, so C is exactly symmetric (the reference's (C+C^T)/2 is
//     a no-op here),
//   * tall-skinny shapes (N >> D, e.g. 401408 x 147 for the ResNet-50 stem)
//     split the row range over blocks; each block stores its fp32 partial
//     tile into a workspace slab and a second kernel sums the slabs in a
//     FIXED split order, applies beta/alpha and writes both triangles.  The
//     result is bitwise reproducible run to run (no float atomics), which
//     the HIP-graph-vs-eager parity test relies on.
//
// Tiling (gfx950, wave64): 128x128 output tile per 256-thread block, 4 waves
// in a 2x2 grid, each wave 64x64 = 2x2 MFMA 32x32 accumulators.  BK = 32
// rows of X per k-tile.  The X tile is staged row-major in LDS ([k][col],
// 320-B rows: conflict-free for the transposed reads) and the MFMA operands
// (8 consecutive k per lane) come from ds_read_b64_tr_b16 (bf16) or plain
// ds_read_b32 (fp32, v_mfma_f32_32x32x2_f32: exact fp32 products).
#include "common.h"
#include "descs.h"

#include <algorithm>
#include <cstdlib>

namespace kfac {

namespace {

constexpr int BM = 128;     // output tile edge
constexpr int BK = 32;      // rows of X per k-tile
constexpr int NT = 256;     // threads per block
constexpr int LDS_W16 = 160;  // bf16 LDS row (128 + 32 pad) = 320 B
constexpr int LDS_W32 = 132;  // fp32 LDS row (128 + 4 pad)

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf16 __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

// position of (i, j), i <= j, in the row-major packed upper triangle of a
// D x D matrix (the layout of comm_pack's triangle wire)
__device__ __forceinline__ int64_t triu_index(int64_t i, int64_t j, int64_t D) {
  return i * D - i * (i - 1) / 2 + (j - i);
}

// upper-triangle tile enumeration: t -> (bi, bj), bi <= bj, row-major
__device__ __forceinline__ void tile_of(int t, int T, int& bi, int& bj) {
  int i = 0, rem = t;
  while (rem >= T - i) {
    rem -= T - i;
    ++i;
  }
  bi = i;
  bj = i + rem;
}

template <typename TIn>
struct Staging;

// ---- bf16 staging: 2 x 16B per thread per operand per k-tile
template <>
struct Staging<bf16_t> {
  v8i16 r[2][2];  // [operand][pass]

  __device__ __forceinline__ static v8i16 load_chunk(
      const uint16_t* __restrict__ X, int64_t ldx, int64_t row, int64_t row_end,
      int64_t col, int64_t K, bool bias, bool vec_ok) {
    v8i16 v;
    if (row < row_end) {
      const uint16_t* p = X + row * ldx + col;
      if (vec_ok && col + 8 <= K) {
        v = *reinterpret_cast<const v8i16*>(p);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int64_t c = col + e;
          short s = 0;
          if (c < K) s = (short)p[e];
          else if (bias && c == K) s = (short)0x3F80;  // bf16(1.0)
          v[e] = s;
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0;
    }
    return v;
  }

  __device__ __forceinline__ void load(const void* Xv, int64_t ldx,
                                       int64_t n0, int64_t row_end, int64_t K,
                                       bool bias, bool vec_ok, int64_t c0i,
                                       int64_t c0j, bool diag) {
    const uint16_t* X = (const uint16_t*)Xv;
    const int t = threadIdx.x;
    const int chunk = t & 15, rloc = t >> 4;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int64_t row = n0 + rloc + 16 * p;
      r[0][p] = load_chunk(X, ldx, row, row_end, c0i + chunk * 8, K, bias,
                           vec_ok);
      if (!diag)
        r[1][p] = load_chunk(X, ldx, row, row_end, c0j + chunk * 8, K, bias,
                             vec_ok);
    }
  }

  __device__ __forceinline__ void store(short* Li, short* Lj, bool diag) {
    const int t = threadIdx.x;
    const int chunk = t & 15, rloc = t >> 4;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      *reinterpret_cast<v8i16*>(Li + (rloc + 16 * p) * LDS_W16 + chunk * 8) =
          r[0][p];
      if (!diag)
        *reinterpret_cast<v8i16*>(Lj + (rloc + 16 * p) * LDS_W16 + chunk * 8) =
            r[1][p];
    }
  }
};

// ---- fp32 staging: 4 x 16B per thread per operand per k-tile
template <>
struct Staging<float> {
  float4 r[2][4];

  __device__ __forceinline__ static float4 load_chunk(
      const float* __restrict__ X, int64_t ldx, int64_t row, int64_t row_end,
      int64_t col, int64_t K, bool bias, bool vec_ok) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < row_end) {
      const float* p = X + row * ldx + col;
      if (vec_ok && col + 4 <= K) {
        v = *reinterpret_cast<const float4*>(p);
      } else {
        float tmp[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t c = col + e;
          tmp[e] = c < K ? p[e] : ((bias && c == K) ? 1.f : 0.f);
        }
        v = make_float4(tmp[0], tmp[1], tmp[2], tmp[3]);
      }
    }
    return v;
  }

  __device__ __forceinline__ void load(const void* Xv, int64_t ldx,
                                       int64_t n0, int64_t row_end, int64_t K,
                                       bool bias, bool vec_ok, int64_t c0i,
                                       int64_t c0j, bool diag) {
    const float* X = (const float*)Xv;
    const int t = threadIdx.x;
    const int chunk = t & 31, rloc = t >> 5;  // 32 chunks of 4 per row, 8 rows
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int64_t row = n0 + rloc + 8 * p;
      r[0][p] = load_chunk(X, ldx, row, row_end, c0i + chunk * 4, K, bias,
                           vec_ok);
      if (!diag)
        r[1][p] = load_chunk(X, ldx, row, row_end, c0j + chunk * 4, K, bias,
                             vec_ok);
    }
  }

  __device__ __forceinline__ void store(float* Li, float* Lj, bool diag) {
    const int t = threadIdx.x;
    const int chunk = t & 31, rloc = t >> 5;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      *reinterpret_cast<float4*>(Li + (rloc + 8 * p) * LDS_W32 + chunk * 4) =
          r[0][p];
      if (!diag)
        *reinterpret_cast<float4*>(Lj + (rloc + 8 * p) * LDS_W32 + chunk * 4) =
            r[1][p];
    }
  }
};

// ---- implicit im2col (K-HIP-2).  A patch row r = (b, oh, ow) and a column
// chunk at k = (i*kw + j)*C + c (C % chunk == 0, so a chunk never straddles
// two taps) read the 16 contiguous bytes at x[b, oh*sh-ph+i, ow*sw-pw+j,
// c..] (zeros outside the image).  Column decode is done once per block.
struct ColTap {
  int c, i, j;
  int bias_chunk;  // 1: the chunk lies at/after column K (bias column / pad)
  int64_t col;
};

__device__ __forceinline__ ColTap decode_col(int64_t col, int64_t K, const ConvGeom& g) {
  ColTap t;
  t.col = col;
  if (col >= K) {
    t.bias_chunk = 1;
    t.c = t.i = t.j = 0;
    return t;
  }
  const int tap = (int)(col / g.C);
  t.c = (int)(col - (int64_t)tap * g.C);
  t.i = tap / g.kw;
  t.j = tap - t.i * g.kw;
  t.bias_chunk = 0;
  return t;
}

// row -> (b, oh*sh - ph, ow*sw - pw); b < 0 marks a row past the end
struct RowPos {
  int64_t b;
  int ih0, iw0;
};

__device__ __forceinline__ RowPos decode_row(int64_t row, int64_t row_end, const ConvGeom& g) {
  RowPos p;
  if (row >= row_end) {
    p.b = -1;
    p.ih0 = p.iw0 = 0;
    return p;
  }
  const int64_t ohw = (int64_t)g.OH * g.OW;
  p.b = row / ohw;
  const int rem = (int)(row - p.b * ohw);
  const int oh = rem / g.OW;
  const int ow = rem - oh * g.OW;
  p.ih0 = oh * g.sh - g.ph;
  p.iw0 = ow * g.sw - g.pw;
  return p;
}

// element offset of a chunk, or -1 when it is zero (padding / past the end)
__device__ __forceinline__ int64_t patch_offset(const RowPos& p, const ColTap& t, const ConvGeom& g) {
  if (p.b < 0 || t.bias_chunk) return -1;
  const int ih = p.ih0 + t.i, iw = p.iw0 + t.j;
  if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) return -1;
  return p.b * g.sB + (int64_t)ih * g.sH + (int64_t)iw * g.sW + t.c;
}

template <typename TIn>
struct PatchStaging;

template <>
struct PatchStaging<bf16_t> {
  v8i16 r[2][2];
  ColTap ti, tj;

  __device__ __forceinline__ void init(int64_t c0i, int64_t c0j, int64_t K, const ConvGeom& g) {
    const int chunk = threadIdx.x & 15;
    ti = decode_col(c0i + chunk * 8, K, g);
    tj = decode_col(c0j + chunk * 8, K, g);
  }

  __device__ __forceinline__ static v8i16 chunk_of(const uint16_t* X, const RowPos& p,
                                                   const ColTap& t, const ConvGeom& g,
                                                   int64_t K, bool bias) {
    v8i16 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0;
    if (p.b >= 0 && t.bias_chunk) {
      if (bias && t.col == K) v[0] = (short)0x3F80;  // bf16(1.0)
      return v;
    }
    const int64_t off = patch_offset(p, t, g);
    if (off >= 0) v = *reinterpret_cast<const v8i16*>(X + off);
    return v;
  }

  __device__ __forceinline__ void load(const void* Xv, int64_t, int64_t n0, int64_t row_end,
                                       int64_t K, bool bias, bool, int64_t, int64_t,
                                       bool diag, const ConvGeom& g) {
    const uint16_t* X = (const uint16_t*)Xv;
    const int rloc = threadIdx.x >> 4;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const RowPos pos = decode_row(n0 + rloc + 16 * p, row_end, g);
      r[0][p] = chunk_of(X, pos, ti, g, K, bias);
      if (!diag) r[1][p] = chunk_of(X, pos, tj, g, K, bias);
    }
  }

  __device__ __forceinline__ void store(short* Li, short* Lj, bool diag) {
    const int t = threadIdx.x;
    const int chunk = t & 15, rloc = t >> 4;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      *reinterpret_cast<v8i16*>(Li + (rloc + 16 * p) * LDS_W16 + chunk * 8) = r[0][p];
      if (!diag)
        *reinterpret_cast<v8i16*>(Lj + (rloc + 16 * p) * LDS_W16 + chunk * 8) = r[1][p];
    }
  }
};

template <>
struct PatchStaging<float> {
  float4 r[2][4];
  ColTap ti, tj;

  __device__ __forceinline__ void init(int64_t c0i, int64_t c0j, int64_t K, const ConvGeom& g) {
    const int chunk = threadIdx.x & 31;
    ti = decode_col(c0i + chunk * 4, K, g);
    tj = decode_col(c0j + chunk * 4, K, g);
  }

  __device__ __forceinline__ static float4 chunk_of(const float* X, const RowPos& p,
                                                    const ColTap& t, const ConvGeom& g,
                                                    int64_t K, bool bias) {
    if (p.b >= 0 && t.bias_chunk)
      return make_float4((bias && t.col == K) ? 1.f : 0.f, 0.f, 0.f, 0.f);
    const int64_t off = patch_offset(p, t, g);
    if (off >= 0) return *reinterpret_cast<const float4*>(X + off);
    return make_float4(0.f, 0.f, 0.f, 0.f);
  }

  __device__ __forceinline__ void load(const void* Xv, int64_t, int64_t n0, int64_t row_end,
                                       int64_t K, bool bias, bool, int64_t, int64_t,
                                       bool diag, const ConvGeom& g) {
    const float* X = (const float*)Xv;
    const int rloc = threadIdx.x >> 5;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const RowPos pos = decode_row(n0 + rloc + 8 * p, row_end, g);
      r[0][p] = chunk_of(X, pos, ti, g, K, bias);
      if (!diag) r[1][p] = chunk_of(X, pos, tj, g, K, bias);
    }
  }

  __device__ __forceinline__ void store(float* Li, float* Lj, bool diag) {
    const int t = threadIdx.x;
    const int chunk = t & 31, rloc = t >> 5;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      *reinterpret_cast<float4*>(Li + (rloc + 8 * p) * LDS_W32 + chunk * 4) = r[0][p];
      if (!diag)
        *reinterpret_cast<float4*>(Lj + (rloc + 8 * p) * LDS_W32 + chunk * 4) = r[1][p];
    }
  }
};

// ---- implicit im2col, 32-bit fast path (fp32 inputs, N < 2^24 rows and an
// input of < 2^31 elements: every ResNet-50 conv).  PMC of the generic
// staging above (profiles/pmc/syrk_r3.md): ~23 VALU instructions per MFMA,
// most of them the two 64-bit divisions of decode_row per row pass and the
// 64-bit patch offsets, so the SIMDs issued VALU, not MFMA.  Here a row is
// decoded with float-reciprocal divisions (one +-1 correction: exact for
// n < 2^24), the tap of each column chunk is folded into one int32 offset at
// init, and a row pass costs one base offset shared by both operands.
__device__ __forceinline__ int fdivmod(int n, int d, float inv, int& r) {
  int q = (int)((float)n * inv);
  r = n - q * d;
  if (r < 0) {
    q -= 1;
    r += d;
  } else if (r >= d) {
    q += 1;
    r -= d;
  }
  return q;
}

struct Tap32 {
  int off;   // i * sH + j * sW + c
  int i, j;  // tap position (bounds)
  int kind;  // 0: image chunk, 1: the bias column (1 at col == K), 2: zero pad
  bool one;  // kind 1 and this chunk holds column K in its first element
};

__device__ __forceinline__ Tap32 tap32(int64_t col, int64_t K, const ConvGeom& g) {
  Tap32 t;
  if (col >= K) {
    t.kind = col == K ? 1 : 2;
    t.one = col == K;
    t.off = t.i = t.j = 0;
    return t;
  }
  const int tap = (int)col / g.C;
  const int c = (int)col - tap * g.C;
  t.i = tap / g.kw;
  t.j = tap - t.i * g.kw;
  t.off = t.i * (int)g.sH + t.j * (int)g.sW + c;
  t.kind = 0;
  t.one = false;
  return t;
}

template <typename TIn>
struct PatchStaging32;

template <>
struct PatchStaging32<float> {
  float4 r[2][4];
  Tap32 ti, tj;
  float inv_ohw, inv_ow;

  __device__ __forceinline__ void init(int64_t c0i, int64_t c0j, int64_t K, const ConvGeom& g) {
    const int chunk = threadIdx.x & 31;
    ti = tap32(c0i + chunk * 4, K, g);
    tj = tap32(c0j + chunk * 4, K, g);
    inv_ohw = 1.f / (float)(g.OH * g.OW);
    inv_ow = 1.f / (float)g.OW;
  }

  __device__ __forceinline__ static float4 chunk_of(const float* X, bool live, int base, int ih0,
                                                    int iw0, const Tap32& t, const ConvGeom& g,
                                                    bool bias) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!live) return v;
    if (t.kind == 0) {
      const int ih = ih0 + t.i, iw = iw0 + t.j;
      if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
        v = *reinterpret_cast<const float4*>(X + (base + t.off));
    } else if (bias && t.one) {
      v.x = 1.f;
    }
    return v;
  }

  __device__ __forceinline__ void load(const void* Xv, int64_t, int64_t n0, int64_t row_end,
                                       int64_t, bool bias, bool, int64_t, int64_t, bool diag,
                                       const ConvGeom& g) {
    const float* X = (const float*)Xv;
    const int rloc = threadIdx.x >> 5;
    const int ohw = g.OH * g.OW;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row = (int)n0 + rloc + 8 * p;
      const bool live = row < (int)row_end;
      int rem, ow;
      const int b = fdivmod(row, ohw, inv_ohw, rem);
      const int oh = fdivmod(rem, g.OW, inv_ow, ow);
      const int ih0 = oh * g.sh - g.ph, iw0 = ow * g.sw - g.pw;
      const int base = b * (int)g.sB + ih0 * (int)g.sH + iw0 * (int)g.sW;
      r[0][p] = chunk_of(X, live, base, ih0, iw0, ti, g, bias);
      if (!diag) r[1][p] = chunk_of(X, live, base, ih0, iw0, tj, g, bias);
    }
  }
};

// ---- implicit im2col on bf16 planes, 32-bit addressing: NPL = 1 (bf16
// input) or 2 (an fp32 input pre-split once into hi / lo bf16 planes by
// split_planes_kernel, so the SYRK loop does no fp32 -> bf16 conversion:
// each input element is otherwise split kh*kw*T times, once per tap and
// column tile that reads it).  Thread t stages one row (t >> 3) of the
// k-tile and the 8-element chunks (t & 7) and (t & 7) + 8 of each operand:
// one row decode per k-tile instead of one per chunk.  Needs C % 8 == 0.
template <int NPL>
struct PatchPlanes32 {
  v8i16 r[2][NPL][2];  // [operand][plane][chunk]
  Tap32 ti[2], tj[2];
  float inv_ohw, inv_ow;

  __device__ __forceinline__ void init(int64_t c0i, int64_t c0j, int64_t K, const ConvGeom& g) {
    const int c = threadIdx.x & 7;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      ti[q] = tap32(c0i + (c + 8 * q) * 8, K, g);
      tj[q] = tap32(c0j + (c + 8 * q) * 8, K, g);
    }
    inv_ohw = 1.f / (float)(g.OH * g.OW);
    inv_ow = 1.f / (float)g.OW;
  }

  // buffer loads: a chunk outside the image (padding), past the last row or
  // in the pad columns gets an offset beyond the descriptor's range, and the
  // hardware returns zeros (no exec masking, no zero-init moves)
  __device__ __forceinline__ static v8i16 chunk_of(__amdgpu_buffer_rsrc_t rs, int poff, bool live,
                                                   int base, int ih0, int iw0, const Tap32& t,
                                                   const ConvGeom& g, bool bias, bool hi_plane) {
    const int ih = ih0 + t.i, iw = iw0 + t.j;
    const bool ok = live && t.kind == 0 && (unsigned)ih < (unsigned)g.H &&
                    (unsigned)iw < (unsigned)g.W;
    const int off = ok ? (base + t.off) * 2 + poff : (int)0x80000000u;
    const v4u32 raw = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    v8i16 v = __builtin_bit_cast(v8i16, raw);
    if (bias && hi_plane && t.one && live) v[0] = (short)0x3F80;  // bf16(1.0)
    return v;
  }

  __device__ __forceinline__ void load(const void* Xv, int64_t, int64_t n0, int64_t row_end,
                                       int64_t, bool bias, bool, int64_t, int64_t, bool diag,
                                       const ConvGeom& g) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(Xv), (short)0, (int)g.nbytes, 0x00020000);
    const int row = (int)n0 + (threadIdx.x >> 3);
    const bool live = row < (int)row_end;
    int rem, ow;
    const int b = fdivmod(row, g.OH * g.OW, inv_ohw, rem);
    const int oh = fdivmod(rem, g.OW, inv_ow, ow);
    const int ih0 = oh * g.sh - g.ph, iw0 = ow * g.sw - g.pw;
    const int base = b * (int)g.sB + ih0 * (int)g.sH + iw0 * (int)g.sW;
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl) {
      const int poff = pl * (int)g.plane * 2;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        r[0][pl][q] = chunk_of(rs, poff, live, base, ih0, iw0, ti[q], g, bias, pl == 0);
        if (!diag) r[1][pl][q] = chunk_of(rs, poff, live, base, ih0, iw0, tj[q], g, bias, pl == 0);
      }
    }
  }

  // plane pl of an operand at L + pl * BK * LDS_W16 (the SPLIT layout)
  __device__ __forceinline__ void store(short* Li, short* Lj, bool diag) {
    const int row = threadIdx.x >> 3, c = threadIdx.x & 7;
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int off = pl * BK * LDS_W16 + row * LDS_W16 + (c + 8 * q) * 8;
        *reinterpret_cast<v8i16*>(Li + off) = r[0][pl][q];
        if (!diag) *reinterpret_cast<v8i16*>(Lj + off) = r[1][pl][q];
      }
  }
};

// dense mode: the existing Staging with the common load signature
template <typename TIn>
struct DenseStaging : Staging<TIn> {
  __device__ __forceinline__ void init(int64_t, int64_t, int64_t, const ConvGeom&) {}
  __device__ __forceinline__ void load(const void* X, int64_t ldx, int64_t n0, int64_t row_end,
                                       int64_t K, bool bias, bool vec_ok, int64_t c0i,
                                       int64_t c0j, bool diag, const ConvGeom&) {
    Staging<TIn>::load(X, ldx, n0, row_end, K, bias, vec_ok, c0i, c0j, diag);
  }
};

// fp32 inputs on bf16 MFMA ("bf16x3"): the staged fp32 tile is split on
// the way into LDS, x = hi + lo (hi = bf16_rn(x), lo = bf16_rn(x - hi)),
// into two bf16 planes per operand, and x_i x_j is accumulated as
// lo.hi + hi.lo + hi.hi -- three 32x32x16 bf16 MFMAs per fragment pair
// instead of eight fp32 32x32x2 MFMAs of the same work, with an error of a
// few 1e-6 relative per product (the dropped lo.lo term and the rounding
// of lo), fp32-class for a covariance.  KFAC_SYRK_FP32=exact keeps the
// exact-product fp32 MFMA path.
__device__ __forceinline__ void split_f4(const float4 v, v4i16& hi, v4i16& lo) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 x01 = {v.x, v.y}, x23 = {v.z, v.w};
  const uint32_t h01 = __builtin_bit_cast(uint32_t, __builtin_convertvector(x01, bf2));
  const uint32_t h23 = __builtin_bit_cast(uint32_t, __builtin_convertvector(x23, bf2));
  const f2 r01 = {v.x - __uint_as_float(h01 << 16), v.y - __uint_as_float(h01 & 0xFFFF0000u)};
  const f2 r23 = {v.z - __uint_as_float(h23 << 16), v.w - __uint_as_float(h23 & 0xFFFF0000u)};
  const uint32_t l01 = __builtin_bit_cast(uint32_t, __builtin_convertvector(r01, bf2));
  const uint32_t l23 = __builtin_bit_cast(uint32_t, __builtin_convertvector(r23, bf2));
  hi = __builtin_bit_cast(v4i16, make_uint2(h01, h23));
  lo = __builtin_bit_cast(v4i16, make_uint2(l01, l23));
}

// Wraps an fp32 staging (dense or implicit-im2col: both hold 4 float4 per
// operand, rows rloc + 8p, columns 4 * (t & 31)) and stores split planes:
// operand base -> hi plane [BK][LDS_W16], lo plane right after it.
template <typename Base>
struct SplitStaging : Base {
  __device__ __forceinline__ void store(short* Li, short* Lj, bool diag) {
    const int t = threadIdx.x;
    const int chunk = t & 31, rloc = t >> 5;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int off = (rloc + 8 * p) * LDS_W16 + chunk * 4;
      v4i16 h, lo;
      split_f4(this->r[0][p], h, lo);
      *reinterpret_cast<v4i16*>(Li + off) = h;
      *reinterpret_cast<v4i16*>(Li + BK * LDS_W16 + off) = lo;
      if (!diag) {
        split_f4(this->r[1][p], h, lo);
        *reinterpret_cast<v4i16*>(Lj + off) = h;
        *reinterpret_cast<v4i16*>(Lj + BK * LDS_W16 + off) = lo;
      }
    }
  }
};

// fp32 NHWC input (any batch / row / pixel strides, channel stride 1) ->
// contiguous NHWC bf16 planes hi = bf16_rn(x), lo = bf16_rn(x - hi)
__global__ void __launch_bounds__(256) split_planes_kernel(
    const float* __restrict__ x, int64_t sB, int64_t sH, int64_t sW, int H, int W, int C,
    int64_t total4, uint16_t* __restrict__ hi, uint16_t* __restrict__ lo) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total4;
       i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * 4;
    const int c = (int)(e % C);
    const int64_t pix = e / C;
    const int w = (int)(pix % W);
    const int64_t bh = pix / W;
    const int h = (int)(bh % H);
    const int64_t b = bh / H;
    const float4 v = *reinterpret_cast<const float4*>(x + b * sB + h * sH + w * sW + c);
    v4i16 vh, vl;
    split_f4(v, vh, vl);
    *reinterpret_cast<v4i16*>(hi + e) = vh;
    *reinterpret_cast<v4i16*>(lo + e) = vl;
  }
}

// bf16 operand fragment for a 32-wide column block `cb` at k offset `kk`:
// lane l gets X[k = kk + 8h + j][col = cb + (l & 31)], j = 0..7, h = l >> 5,
// via two ds_read_b64_tr_b16 (4 k-rows each).
__device__ __forceinline__ v8bf16 frag_bf16(const short* L, int cb, int kk) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4;        // 16-lane group
  const int i = l & 15;        // lane in group: i = 4q + p
  const int q = i >> 2, p = i & 3;
  const int col = cb + 16 * (g & 1) + 4 * p;
  const int krow = kk + 8 * (g >> 1) + q;
  const short* a0 = L + krow * LDS_W16 + col;
  const short* a1 = a0 + 4 * LDS_W16;
  v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)a0);
  v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)a1);
  v8i16 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(v8bf16, c);
}

template <typename TIn, typename Stage, bool SPLIT = false>
__global__ void __launch_bounds__(NT)
syrk_kernel(const void* __restrict__ X, int64_t N, int64_t K, int64_t ldx,
            int bias, float* __restrict__ C, int64_t D, int64_t ldc, int packed,
            float alpha, const float* __restrict__ ascale, float beta, int T, int splits,
            int64_t rows_per_split, int vec_ok, ConvGeom geom, float* __restrict__ ws,
            int xcd_order) {
  constexpr bool F32 = std::is_same<TIn, float>::value && !SPLIT;
  using LT = typename std::conditional<F32, float, short>::type;
  constexpr int LW = F32 ? LDS_W32 : LDS_W16;
  constexpr int PLANES = SPLIT ? 2 : 1;  // bf16 hi (+ lo) planes per operand
  __shared__ __attribute__((aligned(16))) LT lds[2 * PLANES * BK * LW];
  LT* Li = lds;
  LT* Lj = lds + PLANES * BK * LW;

  // XCD-aware order: the dispatcher deals blocks to the 8 XCDs round robin,
  // so XCD x runs blocks x, x + 8, ...  Those take a contiguous run of the
  // (split, tile) order, tiles fastest: the blocks resident on one XCD at a
  // time are the tiles of the same row range, which read the same X rows --
  // from that XCD's L2 after the first tile instead of from HBM
  // (block-per-(tile, split) order left every tile streaming its panels
  // from HBM: L2 hit 0.32, MFMA busy 12.5 %, profiles/pmc/pmc_syrk_r3.md).
  const int tiles = T * (T + 1) / 2;
  const int nblk = tiles * splits;
  const int per_xcd = (nblk + 7) >> 3;
  const int vb = xcd_order ? (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3)
                           : (int)blockIdx.x;
  if (vb >= nblk) return;
  // (xcd_order 0, KFAC_SYRK_XCD_ORDER=0: the round-4 order, tile-major)
  const int split = xcd_order ? vb / tiles : vb % splits;
  const int tile = xcd_order ? vb - split * tiles : vb / splits;
  int bi, bj;
  tile_of(tile, T, bi, bj);
  const bool diag = bi == bj;
  LT* Lb = diag ? Li : Lj;
  const int64_t c0i = (int64_t)bi * BM, c0j = (int64_t)bj * BM;
  const int64_t n_begin = (int64_t)split * rows_per_split;
  int64_t n_end = n_begin + rows_per_split;
  if (n_end > N) n_end = N;

  const int w = threadIdx.x >> 6;
  const int l = threadIdx.x & 63;
  const int wr = w >> 1, wc = w & 1;

  v16f acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  Stage st;
  st.init(c0i, c0j, K, geom);
  const int64_t ntiles = n_end > n_begin ? ceil_div(n_end - n_begin, BK) : 0;
  if (ntiles > 0) {
    st.load(X, ldx, n_begin, n_end, K, bias, vec_ok, c0i, c0j, diag, geom);
    st.store((decltype(&lds[0]))Li, (decltype(&lds[0]))Lj, diag);
    __syncthreads();
  }
  for (int64_t kt = 0; kt < ntiles; ++kt) {
    const bool more = kt + 1 < ntiles;
    if (more)
      st.load(X, ldx, n_begin + (kt + 1) * BK, n_end, K, bias, vec_ok, c0i,
              c0j, diag, geom);
    if constexpr (SPLIT) {
      const short* Lih = (const short*)Li;
      const short* Lil = Lih + BK * LW;
      const short* Lbh = (const short*)Lb;
      const short* Lbl = Lbh + BK * LW;
#pragma unroll
      for (int kk = 0; kk < BK; kk += 16) {
        v8bf16 ah[2], al[2], bh[2], bl[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          ah[q] = frag_bf16(Lih, wr * 64 + 32 * q, kk);
          al[q] = frag_bf16(Lil, wr * 64 + 32 * q, kk);
          bh[q] = frag_bf16(Lbh, wc * 64 + 32 * q, kk);
          bl[q] = frag_bf16(Lbl, wc * 64 + 32 * q, kk);
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[a], bh[b], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bl[b], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bh[b], acc[a][b], 0, 0, 0);
          }
      }
    } else if constexpr (F32) {
      const int h = l >> 5, r = l & 31;
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) {
        float a0 = Li[(kk + h) * LW + wr * 64 + r];
        float a1 = Li[(kk + h) * LW + wr * 64 + 32 + r];
        float b0 = Lb[(kk + h) * LW + wc * 64 + r];
        float b1 = Lb[(kk + h) * LW + wc * 64 + 32 + r];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 16) {
        v8bf16 a0 = frag_bf16((const short*)Li, wr * 64, kk);
        v8bf16 a1 = frag_bf16((const short*)Li, wr * 64 + 32, kk);
        v8bf16 b0 = frag_bf16((const short*)Lb, wc * 64, kk);
        v8bf16 b1 = frag_bf16((const short*)Lb, wc * 64 + 32, kk);
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
      }
    }
    __syncthreads();
    if (more) {
      st.store((decltype(&lds[0]))Li, (decltype(&lds[0]))Lj, diag);
      __syncthreads();
    }
  }

  // ---- epilogue.  C/D layout of a 32x32 MFMA tile: col = lane & 31,
  // row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5).
  // ascale: optional device factor of alpha (the AMP loss-scale correction
  // 1/s^2, read here so the host never waits for the scaler)
  if (ascale != nullptr && splits == 1) alpha *= ascale[0];
  const bool vec_mirror = ((D & 3) == 0) && ((ldc & 3) == 0) &&
                          ((reinterpret_cast<uintptr_t>(C) & 15) == 0);
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) {
      const int64_t gc = c0j + wc * 64 + nj * 32 + (l & 31);
      if (splits > 1) {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const int64_t gr0 = c0i + wr * 64 + mi * 32 + 8 * rb + 4 * (l >> 5);
          // partial tile -> workspace slab [tile][split][BM][BM] (plain
          // stores; 32 lanes write 128 contiguous bytes per row)
          float* slab = ws + ((int64_t)tile * splits + split) * (BM * BM);
          const int lc = wc * 64 + nj * 32 + (l & 31);
          // (rows / columns past D are never read: skip them)
          if (gc < D) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int lr = wr * 64 + mi * 32 + 8 * rb + 4 * (l >> 5) + e;
              if (gr0 + e < D) slab[lr * BM + lc] = acc[mi][nj][rb * 4 + e];
            }
          }
        }
        continue;
      }
      // Read-modify-write of C (the EMA): the 16 old values of this
      // accumulator are loaded together first, at clamped in-bounds
      // addresses (masked when combined), then combined and stored.  (Loaded
      // inside the per-element bounds branch, each load was waited for
      // alone: 64 dependent round trips per lane per tile.)
      float old[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) old[q] = 0.f;
      if (beta != 0.f) {
        const int64_t gcc = gc < D ? gc : D - 1;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int64_t gr = c0i + wr * 64 + mi * 32 + 8 * (q >> 2) + 4 * (l >> 5) + (q & 3);
          const int64_t grc = gr < D ? gr : D - 1;
          int64_t idx;
          if (packed) idx = grc <= gcc ? triu_index(grc, gcc, D) : 0;
          else idx = grc * ldc + gcc;
          old[q] = C[idx];
        }
      }
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const int64_t gr0 = c0i + wr * 64 + mi * 32 + 8 * rb + 4 * (l >> 5);
        if (packed) {
          // packed upper triangle (the all-reduce wire layout): owned
          // elements only, read-modify-write in place, no mirror
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int64_t gr = gr0 + e;
            if (gr < D && gc < D && gr <= gc) {
              const int64_t pi = triu_index(gr, gc, D);
              C[pi] = beta * old[rb * 4 + e] + alpha * acc[mi][nj][rb * 4 + e];
            }
          }
        } else if (!diag) {
          // strictly upper tile: write C[gr][gc] and mirror C[gc][gr..gr+3]
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int64_t gr = gr0 + e;
            v[e] = beta * old[rb * 4 + e] + alpha * acc[mi][nj][rb * 4 + e];
            if (gr < D && gc < D) C[gr * ldc + gc] = v[e];
          }
          if (gc < D) {
            if (vec_mirror && gr0 + 3 < D) {
              *reinterpret_cast<float4*>(&C[gc * ldc + gr0]) =
                  make_float4(v[0], v[1], v[2], v[3]);
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (gr0 + e < D) C[gc * ldc + gr0 + e] = v[e];
            }
          }
        } else {
          // diagonal tile: own the upper half, mirror it
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int64_t gr = gr0 + e;
            if (gr < D && gc < D && gr <= gc) {
              const float v = beta * old[rb * 4 + e] + alpha * acc[mi][nj][rb * 4 + e];
              C[gr * ldc + gc] = v;
              if (gr != gc) C[gc * ldc + gr] = v;
            }
          }
        }
      }
    }
  }
}

// Split-K reduction: one 32x32 sub-block of the upper triangle per block.
// C[i][j] = beta*C[i][j] + alpha * sum_s slab[s][i][j]  (s ascending), and
// C[j][i] = C[i][j] through an LDS transpose (both writes coalesced).
// Two passes when the triangle has too few sub-blocks to fill the chip
// (D = 64 with 512 slabs: 3 blocks, 30-120 us in the r3 step trace):
// pass 1, grid (sub-blocks, groups), sums the `count` slabs of one group
// (slabs g*gs .. g*gs+count-1, ascending) back into slab g*gs; pass 2
// (final) sums the group slabs 0, gs, 2gs, ... in order.  The summation
// order is fixed by (splits, gs) alone, so results stay bitwise
// reproducible run to run.
__global__ void __launch_bounds__(256)
splitk_reduce_kernel(float* __restrict__ ws, int splits, int T, int gs, int final_pass,
                     float* __restrict__ C, int64_t D, int64_t ldc, int packed,
                     float alpha, const float* __restrict__ ascale, float beta, int T32) {
  if (ascale != nullptr) alpha *= ascale[0];
  __shared__ float tile[32][33];
  // blockIdx.x -> (bi, bj), bi <= bj, over the T32 x T32 sub-block grid
  int bi, bj;
  tile_of((int)blockIdx.x, T32, bi, bj);
  const int t = threadIdx.x;
  const int r = t >> 3, c4 = (t & 7) * 4;
  const int ti = bi >> 2, tj = bj >> 2;
  const int64_t tidx = (int64_t)ti * T - (int64_t)ti * (ti - 1) / 2 + (tj - ti);
  const int lr = (bi & 3) * 32 + r, lc = (bj & 3) * 32 + c4;
  // pass 1: slabs g*gs + u (u < count); final: slabs u*gs (u < count)
  const int g = (int)blockIdx.y;
  const int first = final_pass ? 0 : g * gs;
  const int count = final_pass ? (int)ceil_div(splits, gs) : min(gs, splits - first);
  const int64_t step = (int64_t)(final_pass ? gs : 1) * (BM * BM);
  float* src = ws + (tidx * splits + first) * (BM * BM) + lr * BM + lc;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  // 8 independent loads in flight per thread (fixed summation order)
  int s = 0;
  for (; s + 8 <= count; s += 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = *reinterpret_cast<const float4*>(src + (int64_t)(s + u) * step);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      acc.x += v[u].x;
      acc.y += v[u].y;
      acc.z += v[u].z;
      acc.w += v[u].w;
    }
  }
  for (; s < count; ++s) {
    const float4 v = *reinterpret_cast<const float4*>(src + (int64_t)s * step);
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  if (!final_pass) {
    *reinterpret_cast<float4*>(src) = acc;
    return;
  }
  const int64_t gr = (int64_t)bi * 32 + r;
  const float a4[4] = {acc.x, acc.y, acc.z, acc.w};
  // the EMA's old values, loaded together (clamped addresses) before any
  // store: one memory round trip instead of four dependent ones
  bool upper[4];
  int64_t idx[4];
  float old[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t gc = (int64_t)bj * 32 + c4 + e;
    upper[e] = gr < D && gc < D && (bi < bj || gr <= gc);
    idx[e] = upper[e] ? (packed ? triu_index(gr, gc, D) : gr * ldc + gc) : 0;
    if (beta != 0.f) old[e] = C[idx[e]];
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float v = 0.f;
    if (upper[e]) {
      v = beta * old[e] + alpha * a4[e];
      C[idx[e]] = v;
    }
    tile[r][c4 + e] = v;
  }
  if (packed) return;  // uniform: the packed triangle has no mirror
  __syncthreads();
  // mirror: C[bj*32 + r][bi*32 + c] = tile[c][r]  (strictly lower elements)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = c4 + e;
    const int64_t i = (int64_t)bj * 32 + r, j = (int64_t)bi * 32 + c;
    if (i < D && j < D && j < i) C[i * ldc + j] = tile[c][r];
  }
}

}  // namespace

// Row splits for one SYRK.  Only shapes whose upper-triangle tile count
// cannot fill the chip are split (target ~128 blocks), and the fp32
// partial-tile workspace is capped at 32 MB.
int64_t syrk_workspace_splits(int64_t N, int64_t D) {
  const int64_t T = ceil_div(D, BM);
  const int64_t tiles = T * (T + 1) / 2;
  // KFAC_SYRK_TARGET_BLOCKS (default 128): the factor SYRKs run beside
  // backward on the factor stream, where fewer, longer blocks cost the
  // overlapped step less than filling the chip does.  ResNet-50 bench
  // factor step: 768 -> 22.7 ms, 256 -> 21.3, 128 -> 20.6-20.7, 96 -> 20.9,
  // 64 -> 24.1 (profiles/r5/syrk_target_ab/)
  static const int64_t target_blocks = [] {
    const char* e = std::getenv("KFAC_SYRK_TARGET_BLOCKS");
    const long v = e != nullptr ? std::atol(e) : 0;
    return (int64_t)(v > 0 ? v : 128);
  }();
  int64_t splits = ceil_div(target_blocks, tiles);
  const int64_t max_by_rows = ceil_div(N, 4 * BK);  // >= 4 k-tiles per split
  if (splits > max_by_rows) splits = max_by_rows;
  const int64_t max_by_ws = (int64_t(32) << 20) / (4 * tiles * BM * BM);
  if (splits > max_by_ws) splits = max_by_ws;
  // the reduction re-reads every slab once: beyond ~64 slabs per tile it
  // costs more than the extra parallelism gains (PMC: profiles/pmc) --
  // unless the triangle has so few tiles that 64 splits cannot fill the
  // chip (the 147-wide A factor of ResNet's 7x7 stem: 3 tiles x 64 splits
  // = 192 blocks for 401k rows)
  // KFAC_SYRK_ONE_TILE_SPLITS: the cap for a one-tile triangle (D <= 128:
  // the 64-channel G factors, 100k-400k rows), whose blocks are otherwise
  // a latency-bound chain of ~200 k-tiles each
  static const int64_t one_tile_cap = [] {
    const char* e = std::getenv("KFAC_SYRK_ONE_TILE_SPLITS");
    const long v = e != nullptr ? std::atol(e) : 0;
    return (int64_t)(v > 0 ? v : 64);
  }();
  int64_t cap = tiles * 64 >= target_blocks / 2 ? 64 : ceil_div(target_blocks, tiles);
  if (tiles == 1 && one_tile_cap > cap) {
    cap = one_tile_cap;
    splits = std::min<int64_t>(one_tile_cap, std::min(max_by_rows, max_by_ws));
  }
  if (splits > cap) splits = cap;
  if (splits < 2) splits = 1;
  return splits;
}

int64_t syrk_workspace_floats(int64_t D, int64_t splits) {
  if (splits <= 1) return 0;
  const int64_t T = ceil_div(D, BM);
  return T * (T + 1) / 2 * splits * BM * BM;
}

// fp32 NHWC conv input -> contiguous bf16 hi / lo planes (hi at `planes`,
// lo at planes + B*H*W*C) for the pre-split implicit-im2col SYRK
void syrk_split_planes(const float* x, int64_t B, int H, int W, int C, int64_t sB, int64_t sH,
                       int64_t sW, uint16_t* planes, hipStream_t s) {
  const int64_t total = B * H * W * (int64_t)C;
  if (total == 0) return;
  const int64_t total4 = total / 4;
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(total4, 256), 8192);
  split_planes_kernel<<<dim3(blocks), dim3(256), 0, s>>>(x, sB, sH, sW, H, W, C, total4, planes,
                                                         planes + total);
}

// geom == nullptr: X is a dense [N, K] matrix (row stride ldx); otherwise
// X is an NHWC conv input and its rows are the conv patches (implicit im2col).
// ws: syrk_workspace_floats(D, splits) floats when splits > 1.
// ldc == 0: C is the packed upper triangle (D (D + 1) / 2 floats, row-major,
// the all-reduce wire layout) and only it is written.
void syrk(int in_dtype, const void* x, int64_t N, int64_t K, int64_t ldx,
          bool bias, float* C, int64_t D, int64_t ldc, float alpha,
          float beta, int splits, hipStream_t s, const ConvGeom* geom,
          float* ws, const float* ascale, bool fp32_exact) {
  const int packed = ldc == 0 ? 1 : 0;
  if (D <= 0) return;
  const int T = (int)ceil_div(D, BM);
  const int64_t tiles = (int64_t)T * (T + 1) / 2;
  if (splits < 1 || ws == nullptr) splits = 1;
  const int64_t rows_per_split =
      splits > 1 ? ceil_div(ceil_div(N, splits), BK) * BK : (N > 0 ? N : 1);
  static const int xcd = [] {
    const char* e = std::getenv("KFAC_SYRK_XCD_ORDER");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
  }();
  // padded to a multiple of the 8 XCDs (syrk_kernel's block order)
  const dim3 grid((unsigned)(8 * ceil_div(tiles * splits, (int64_t)8)));
  ConvGeom g = geom != nullptr ? *geom : ConvGeom{};
  if (geom != nullptr) {
    // bytes the implicit-im2col buffer loads may touch (bf16 elements: the
    // planes, or the bf16 input's last element + 1)
    const int64_t nb = N / ((int64_t)g.OH * g.OW);
    g.nbytes = g.plane > 0 ? 4 * g.plane
                           : 2 * ((nb - 1) * g.sB + (int64_t)(g.H - 1) * g.sH +
                                  (int64_t)(g.W - 1) * g.sW + g.C);
  }
  if (in_dtype == kF32) {
    const int vec_ok = ((ldx & 3) == 0) &&
                       ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
#define SYRK_F32(STAGE, SPLIT_)                                                     \
  syrk_kernel<float, STAGE, SPLIT_><<<grid, dim3(NT), 0, s>>>(                      \
      x, N, K, ldx, bias ? 1 : 0, C, D, ldc, packed, alpha, ascale, beta, T, splits, \
      rows_per_split, vec_ok, g, ws, xcd)
    if (geom != nullptr && g.plane > 0) {
      // pre-split bf16 planes (syrk_split_planes)
      SYRK_F32(PatchPlanes32<2>, true);
    } else if (geom != nullptr) {
      // 32-bit patch addressing when every row index and input offset fits
      // (fdivmod is exact below 2^24 rows)
      const int64_t in_elems = (int64_t)(N / ((int64_t)g.OH * g.OW) + 1) * g.sB;
      const bool fast = N < (int64_t(1) << 24) && in_elems < (int64_t(1) << 31) &&
                        g.sB < (int64_t(1) << 31);
      if (fp32_exact) SYRK_F32(PatchStaging<float>, false);
      else if (fast) SYRK_F32(SplitStaging<PatchStaging32<float>>, true);
      else SYRK_F32(SplitStaging<PatchStaging<float>>, true);
    } else {
      if (fp32_exact) SYRK_F32(DenseStaging<float>, false);
      else SYRK_F32(SplitStaging<DenseStaging<float>>, true);
    }
#undef SYRK_F32
  } else {
    const int vec_ok = ((ldx & 7) == 0) &&
                       ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
    const bool fast32 = geom != nullptr && N < (int64_t(1) << 24) && g.C % 8 == 0 &&
                        g.nbytes < (int64_t(1) << 31) &&
                        (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    if (geom != nullptr && fast32)
      syrk_kernel<bf16_t, PatchPlanes32<1>><<<grid, dim3(NT), 0, s>>>(
          x, N, K, ldx, bias ? 1 : 0, C, D, ldc, packed, alpha, ascale, beta, T, splits,
          rows_per_split, vec_ok, g, ws, xcd);
    else if (geom != nullptr)
      syrk_kernel<bf16_t, PatchStaging<bf16_t>><<<grid, dim3(NT), 0, s>>>(
          x, N, K, ldx, bias ? 1 : 0, C, D, ldc, packed, alpha, ascale, beta, T, splits,
          rows_per_split, vec_ok, g, ws, xcd);
    else
      syrk_kernel<bf16_t, DenseStaging<bf16_t>><<<grid, dim3(NT), 0, s>>>(
          x, N, K, ldx, bias ? 1 : 0, C, D, ldc, packed, alpha, ascale, beta, T, splits,
          rows_per_split, vec_ok, g, ws, xcd);
  }
  if (splits > 1) {
    const int T32 = (int)ceil_div(D, 32);
    const unsigned blocks = (unsigned)((int64_t)T32 * (T32 + 1) / 2);
    // groups for pass 1: enough blocks to fill the chip, <= 16 group slabs
    // for the final pass, >= 4 slabs per group
    // (gs = 1: no pass 1, the final pass sums every slab)
    int gs = 1;
    // (a second launch only pays when one pass would take > ~16 rounds of
    // 8 loads per thread: measured 25 -> 31 us for 49 slabs, 59 -> 45 us
    // for 512, profiles/syrk_probe_r3_v2.jsonl)
    if (blocks < 512 && splits >= 128) {
      int groups = (int)std::min<int64_t>(ceil_div(512, blocks), splits / 4);
      groups = std::max(groups, (int)ceil_div(splits, 64));
      gs = (int)ceil_div(splits, groups);
    }
    if (gs > 1) {
      const unsigned groups = (unsigned)ceil_div(splits, gs);
      splitk_reduce_kernel<<<dim3(blocks, groups), dim3(256), 0, s>>>(
          ws, splits, T, gs, 0, C, D, ldc, packed, alpha, ascale, beta, T32);
    }
    splitk_reduce_kernel<<<dim3(blocks), dim3(256), 0, s>>>(
        ws, splits, T, gs, 1, C, D, ldc, packed, alpha, ascale, beta, T32);
  }
}

}  // namespace kfac
