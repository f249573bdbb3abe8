// Device descriptor tables shared by the multi-tensor kernels and the
// bindings (one definition; the bindings pack them on the host).
#pragma once
#include <cstdint>

namespace kfac {

// multi.hip: one K-FAC layer of the KL-clip / apply launches
struct LayerDesc {
  const float* p;   // preconditioned grad [rows, cols], row stride ldp
  void* w;          // weight grad [rows, wcols] contiguous
  void* b;          // bias grad [rows] or null
  int64_t rows, cols, ldp, wcols;
  int64_t block_start;  // first block of this layer
  int32_t wdt, bdt;     // dtype tags
  // weight of the bias term in the KL sum: 1, or 1/mp for a bias replicated
  // over the mp ranks of a row-parallel (tensor-parallel) layer, so an
  // all-reduce of the per-rank sums counts it once
  float bscale;
  int32_t pad;
};

// gemm3.hip: one GEMM of a grouped launch
struct GemmDesc {
  const float* A;        // A storage: [M][lda] (k-contig) or [K][lda] (m-contig)
  const float* A_extra;  // optional column Kmain of A (k-contig only): [M]
  const float* B;        // B storage: [K][ldb] (n-contig) or [N][ldb] (k-contig)
  float* C;              // [M][ldc]
  const float* S;        // optional scale matrix [M][lds]
  const float* dg;       // optional scale vectors: C = acc / (dg[m]*da[n] + damping)
  const float* da;
  int64_t lda, ldb, ldc, lds;
  int32_t M, N, K, Kmain;
  int32_t tiles_n, tile_start;
  float damping;
  int32_t vec;  // bit0: A float4 loads ok, bit1: B float4 loads ok
  // optional pre-split operands: x = hi + lo (bf16) computed once per
  // second-order update (the eigenbases are constant between updates),
  // interleaved per 4 elements in the fp32 operand's layout, so the kernel
  // stores them to LDS without the per-tile split
  const uint16_t* Ah;
  const uint16_t* Bh;
  // optional BatchNorm statistics of the output (single-pass GEMMs without
  // an epilogue scaling): per 64-row half tile and column, the sum and the
  // sum of squares of the stored values, [2 * tiles_m][2][N] fp32 -- the
  // partials the fused BN's finalize reads (csrc/bnact.hip), so the BN that
  // follows a native convolution skips its statistics pass
  float* bnpart;
  // optional addend [M][ldc] added to the stored values (may alias C: an
  // accumulation of the GEMM into an existing gradient)
  const float* D;
};

// gemm3s.hip: one GEMM of a grouped launch on split images.  A split image
// holds a logical matrix as two bf16 planes (hi at the base, lo `plane`
// elements later), each [R][ld] with R and ld multiples of 256 and the
// padding zero, so no load of a 128 x 32 tile ever needs a bounds check.
//   C[M][N] = A[M][K] B[K][N] (K a multiple of 32 or zero-padded to it);
//   A image [M][K] (k-contig) or [K][M] (m-contig); B [N][K] or [K][N].
struct Gemm3sDesc {
  const uint16_t* A;
  const uint16_t* B;
  void* C;              // fp32 [M][ldc], or a split image (hi, lo at +c_plane)
  const float* S;       // optional scale matrix [M][lds]
  const float* dg;      // optional: C = acc / (dg[m] * da[n] + damping)
  const float* da;
  int64_t a_plane, b_plane, c_plane;
  int64_t lda, ldb, ldc, lds;
  int32_t M, N, K;
  int32_t tiles_n, tile_start;
  float damping;
};

// gemm3s.hip: fp32 [rows][cols] (+ one extra column read from a vector)
// -> split image planes at dst (row stride ldd, lo plane at +plane)
struct SplitDesc {
  const float* src;
  const float* extra;
  uint16_t* dst;
  int64_t lds, ldd, plane;
  int64_t block_start;
  int32_t rows, cols;
  int32_t vec;  // src rows 16-B aligned (float4 loads)
  int32_t pad;
};

// syrk.hip implicit-im2col mode: the SYRK input rows are the patches of an
// NHWC conv input, columns in natural (kh, kw, c) order, read straight from
// the activation (the patch matrix is never materialised)
struct ConvGeom {
  int64_t sB, sH, sW;  // element strides of the input (channel stride 1)
  int32_t H, W, C, kw, sh, sw, ph, pw, OH, OW;
  int64_t plane;   // > 0: x holds two bf16 planes (hi, lo) this many elements apart
  int64_t nbytes;  // set by syrk(): bytes the buffer loads may read
};

// sytrd.hip: one matrix of a batched mixed-size tridiagonalisation
struct SytrdDesc {
  float* A;      // [n][n] row-major, full symmetric on entry
  float* Wt;     // [NB][n] panel W, row j = column j of LAPACK's W
  float* d;      // [n]
  float* e;      // [n-1]
  float* tau;    // [n-1]
  float* part1;  // [SY_MAXCH][SY_P1] col-step partials
  float* part2;  // [SY_MAXROWBLK] symv partial w.v
  float* sc;     // [4 + 2 NB]: tau, v scale, t1.t2 of the last reflector,
                 // then t1 = W^T v and t2 = V^T v (tile symv)
  float* P;      // unused (was the tile symv's row partials; layout kept)
  int32_t n, pad;
};

// multi-tensor dtype cast (csrc/cast.hip): one tensor's storage-order
// elements, fp32 <-> bf16
struct CastDesc {
  const void* src;
  void* dst;
  int64_t n;            // elements
  int64_t block_start;  // first block of this tensor in the launch
  int32_t vec;          // both pointers 16-B aligned: 8-element vector path
  int32_t pad;
};

}  // namespace kfac
