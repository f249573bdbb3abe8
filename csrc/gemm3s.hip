// K-HIP-4 v2: grouped bf16x3 GEMM on PRE-SPLIT operands, staged global ->
// LDS by LDS-DMA (global_load_lds_dwordx4).
//
// The per-step K-FAC preconditioning chain (reference kfac/layers/eigen.py:
// 349-384, kfac/layers/inverse.py:214-233) is four dependent fp32 GEMMs per
// layer.  v1 (gemm3.hip) loads fp32 operands into registers, splits every
// element into bf16 hi + lo (x = hi + lo) and writes both to LDS.  Measured
// on the GPT-NeoX-125M T1 set (tools/gemm3_bench.cpp, DIAG builds): with the
// MFMAs removed the kernel takes 93 % of its full time -- the register
// staging + split + ds_write pass, not the matrix cores, is the bound.
//
// v2 removes that pass: every operand already lives in a "split image" --
// two bf16 planes (hi, lo) of the logical matrix, zero-padded to multiples of
// 256 in both dimensions -- so the kernel is a plain bf16 GEMM that issues
// three MFMAs (lo.hi + hi.lo + hi.hi) per fragment pair:
//   * static operands (the eigenbases QA / QG, or the damped inverses) are
//     split once per second-order update;
//   * the weight gradient [Wg | bg] is split by one multi-tensor launch per
//     step (split_pad_multi below; the bias column is appended there, and the
//     zero k-padding removes every bounds check from the K loop);
//   * every intermediate (t1, t2, t3) is written split by the producing
//     GEMM's epilogue, straight into the next GEMM's operand image.
// Bytes per element are unchanged (2 x bf16 = 1 x fp32), but a tile now goes
// global -> LDS with no VGPR round trip and no VALU work: 8 x 16-B DMA
// instructions per wave per k-tile, one plane per wave.
//
// LDS images (per stage: A hi, A lo, B hi, B lo; 8 KiB each):
//   k-contiguous operand ([rows][K]): [128 rows][32 k] with 64-B rows, 16-B
//     chunks XOR-swizzled by (row >> 2) & 3 -> MFMA fragments by ds_read_b128
//     are bank-conflict free over all four 16-lane groups;
//   m-contiguous operand ([K][rows]): [32 k][128 rows] with 256-B rows,
//     chunks swizzled by (k & 3) << 2 -> the transposing ds_read_b64_tr_b16
//     fragment reads hit 32 distinct 8-B slots per half-wave.
// LDS-DMA writes lane-linear, so the swizzle is applied to the SOURCE address
// of each lane and the same involution to the read address.
//
// Tiling (GEMM3S_TILE below): 256x256 output tile per 512-thread block
// (8 waves 2x4, 128x64 each = 4x2 MFMA 32x32x16 accumulators), BK = 32, two
// LDS stages (128 KiB), one block per CU.  XCD-aware chunked tile order and per-layer grouped tile
// rows as v1.  Epilogues: eigenvalue scaling (S = dGdA, or 1/(dG dA^T +
// damping)), then either fp32 (the preconditioned gradient P) or the split
// image of the result (the next GEMM's operand).
#include "common.h"
#include "descs.h"

namespace kfac {

namespace {

constexpr int SK = 32;              // k per stage
#ifndef GEMM3S_CH
#define GEMM3S_CH 4
#endif
#ifndef GEMM3S_GM
#define GEMM3S_GM 8
#endif
constexpr int CH = GEMM3S_CH;
constexpr int GM = GEMM3S_GM;
// diagnostic builds only (tools/gemm3s_bench.cpp): 1 = no DMA, 3 = no MFMA,
// 4 = no epilogue stores
#ifndef GEMM3S_DIAG
#define GEMM3S_DIAG 0
#endif

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf16 __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
typedef const void __attribute__((address_space(1)))* gvoid_t;
typedef void __attribute__((address_space(3)))* lvoid_t;

#define GLOBAL __attribute__((address_space(1)))

__device__ __forceinline__ int find_tile_layer(const Gemm3sDesc* d, int n, int t) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].tile_start <= t) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// One 16-B LDS-DMA wave instruction: lane l's 16 bytes at g land at LDS
// address dst + 16 l.  Issued from inline asm, not the builtin: the builtin
// tells the compiler the instruction writes LDS, and its wait-count pass
// then put an `s_waitcnt vmcnt(0)` in front of the first LDS read after it --
// every k tile waited for the DMA of the NEXT tile before computing the
// current one (the stage pipeline ran fully serialised; PMC: 28 % MFMA busy,
// profiles/r5/pmc/g3s.md).  The stages are ordered by the explicit counted
// waits + barrier at the top of the k loop instead.  m0 (the LDS base) is
// saved and restored around the instruction.
__device__ __forceinline__ void lds_dma16(const uint16_t* g, uint16_t* dst) {
  const uint32_t la = (uint32_t)(uintptr_t)(lvoid_t)dst;
  uint32_t saved;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(saved)
      : "v"((uint64_t)(uintptr_t)g), "s"(__builtin_amdgcn_readfirstlane(la))
      : "memory");
}

// One 16-B LDS-DMA wave-instruction (1 KiB) of an operand plane of one
// stage.  k-contig plane [E rows][32 k] (64-B rows): instruction i covers
// rows 16i..16i+15, chunk c of row r lands at slot c ^ ((r >> 2) & 3).
// m-contig plane [32 k][E cols] (2E-byte rows): instruction i covers bytes
// [1024 i, 1024 i + 1024), chunk c of k-row r at slot c ^ ((r & 3) << 2).
template <bool MC, int E>
__device__ __forceinline__ void stage_instr(const uint16_t* __restrict__ src, int64_t ld,
                                            int org, int k0, uint16_t* plane, int i) {
  const int L = threadIdx.x & 63;
  const uint16_t* g;
  if constexpr (!MC) {
    const int r = 16 * i + (L >> 2);
    const int c = (L & 3) ^ ((r >> 2) & 3);
    g = src + (int64_t)(org + r) * ld + k0 + c * 8;
  } else {
    constexpr int CPR = E / 8;           // 16-B chunks per k-row
    const int flat = 64 * i + L;         // chunk index in the plane
    const int r = flat / CPR;
    const int c = (flat % CPR) ^ ((r & 3) << 2);
    g = src + (int64_t)(k0 + r) * ld + org + c * 8;
  }
  lds_dma16(g, plane + i * 512);
}

// k-contig fragment: lane l gets X[row = base + (l & 31)][k = 16 kh + 8 (l >> 5) + 0..7]
__device__ __forceinline__ v8bf16 frag_kc(const uint16_t* P, int base, int kh) {
  const int l = threadIdx.x & 63;
  const int r = base + (l & 31);
  const int c = (2 * kh + (l >> 5)) ^ ((r >> 2) & 3);
  const v8i16 v = *reinterpret_cast<const v8i16*>(P + r * SK + c * 8);
  return __builtin_bit_cast(v8bf16, v);
}

// m-contig fragment from a [32 k][E] plane: lane l gets
// X[k = 16 kh + 8 (l >> 5) + j][row = base + (l & 31)] through two
// transposing 8-byte reads (4 k-rows each)
template <int E>
__device__ __forceinline__ v8bf16 frag_mc(const uint16_t* P, int base, int kh) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4;
  const int i = l & 15;
  const int q = i >> 2, p = i & 3;
  const int col = base + 16 * (g & 1) + 4 * p;
  const int krow = 16 * kh + 8 * (g >> 1) + q;
  const int chunk = (col >> 3) ^ ((krow & 3) << 2);
  const uint16_t* a0 = P + krow * E + chunk * 8 + (col & 7);
  const uint16_t* a1 = a0 + 4 * E;  // krow + 4: same (krow & 3) swizzle
  v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)a0);
  v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)a1);
  v8i16 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(v8bf16, c);
}

// wait until at most N of this wave's vector-memory operations (LDS-DMA
// included) are outstanding
#define KFAC_VMCNT(n) \
  if constexpr (N == n) { asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); return; }
template <int N>
__device__ __forceinline__ void wait_vm() {
  KFAC_VMCNT(0) KFAC_VMCNT(2) KFAC_VMCNT(3) KFAC_VMCNT(4) KFAC_VMCNT(6) KFAC_VMCNT(8)
  KFAC_VMCNT(12) KFAC_VMCNT(16)
  static_assert(N == 0 || N == 2 || N == 3 || N == 4 || N == 6 || N == 8 || N == 12 || N == 16,
                "unsupported vmcnt");
}
#undef KFAC_VMCNT

__device__ __forceinline__ void split1(float x, uint16_t& hi, uint16_t& lo) {
  const __bf16 h = (__bf16)x;
  hi = __builtin_bit_cast(uint16_t, h);
  const float r = x - (float)h;
  lo = __builtin_bit_cast(uint16_t, (__bf16)r);
}

// BM x BN output tile, WM x WN waves, each wave (BM / WM) x (BN / WN) =
// FM x FN MFMA 32x32 accumulators.
template <int BM, int BN, int WM, int WN, int NSTAGE, bool A_MC, bool B_MC, bool OUT_SPLIT>
__global__ void __launch_bounds__(WM * WN * 64)
gemm3s_kernel(const Gemm3sDesc* __restrict__ descs, int nlayers, int total_tiles) {
  constexpr int NW = WM * WN;
  constexpr int FM = BM / WM / 32, FN = BN / WN / 32;
  constexpr int PA = BM * SK, PB = BN * SK;          // plane elements
  constexpr int STAGE = 2 * PA + 2 * PB;
  constexpr int IA = BM / 16, IB = BN / 16;           // DMA instructions per plane
  constexpr int ITOT = 2 * IA + 2 * IB;
  static_assert(ITOT % NW == 0, "DMA instructions must divide over the waves");
  constexpr int IPW = ITOT / NW;
  __shared__ __attribute__((aligned(16))) uint16_t lds[NSTAGE * STAGE];

  const int b = blockIdx.x;
  const int xcd = b & 7, rr = b >> 3;
  const int t = ((rr / CH) * 8 + xcd) * CH + (rr % CH);
  if (t >= total_tiles) return;
  const Gemm3sDesc d = descs[find_tile_layer(descs, nlayers, t)];
  const int tl = t - d.tile_start;
  const int tiles_m = (d.M + BM - 1) / BM;
  const int per_group = GM * d.tiles_n;
  const int first_m = (tl / per_group) * GM;
  const int gm = min(tiles_m - first_m, GM);
  const int in_group = tl % per_group;
  const int m0 = (first_m + in_group % gm) * BM;
  const int n0 = (in_group / gm) * BN;

  const int w = threadIdx.x >> 6;
  const int l = threadIdx.x & 63;
  const int wr = w / WN, wc = w % WN;

  auto stage = [&](int kt) {
    if constexpr (GEMM3S_DIAG == 1) return;
    uint16_t* base = lds + (kt % NSTAGE) * STAGE;
    const int k0 = kt * SK;
#pragma unroll
    for (int j = 0; j < IPW; ++j) {
      const int idx = w * IPW + j;  // wave-uniform
      if (idx < 2 * IA) {
        const int pl = idx / IA, i = idx % IA;
        const uint16_t* src = d.A + (pl ? d.a_plane : 0);
        stage_instr<A_MC, BM>(src, d.lda, m0, k0, base + pl * PA, i);
      } else {
        const int pl = (idx - 2 * IA) / IB, i = (idx - 2 * IA) % IB;
        const uint16_t* src = d.B + (pl ? d.b_plane : 0);
        stage_instr<B_MC, BN>(src, d.ldb, n0, k0, base + 2 * PA + pl * PB, i);
      }
    }
  };

  v16f acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nt = (d.K + SK - 1) / SK;
  // NSTAGE - 1 k-tiles in flight.  With NSTAGE == 2 the wait + barrier at
  // the end of each k-tile is the plain double buffer; with NSTAGE == 3 the
  // next-but-one tile's DMA stays in flight across the barrier (counted
  // vmcnt, raw s_barrier: __syncthreads would drain every LDS-DMA).
  stage(0);
  if (NSTAGE > 2 && nt > 1) stage(1);
  for (int kt = 0; kt < nt; ++kt) {
    if constexpr (NSTAGE > 2) {
      if (kt + 1 < nt) wait_vm<IPW>();
      else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    // every wave's DMA of tile kt has landed and every wave is done reading
    // the buffer about to be refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + NSTAGE - 1 < nt) stage(kt + NSTAGE - 1);
    const uint16_t* cur = lds + (kt % NSTAGE) * STAGE;
    const uint16_t* Ah = cur;
    const uint16_t* Al = cur + PA;
    const uint16_t* Bh = cur + 2 * PA;
    const uint16_t* Bl = cur + 2 * PA + PB;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      v8bf16 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int am = wr * (BM / WM) + i * 32;
        if constexpr (A_MC) {
          ah[i] = frag_mc<BM>(Ah, am, kh);
          al[i] = frag_mc<BM>(Al, am, kh);
        } else {
          ah[i] = frag_kc(Ah, am, kh);
          al[i] = frag_kc(Al, am, kh);
        }
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int bn = wc * (BN / WN) + j * 32;
        if constexpr (B_MC) {
          bh[j] = frag_mc<BN>(Bh, bn, kh);
          bl[j] = frag_mc<BN>(Bl, bn, kh);
        } else {
          bh[j] = frag_kc(Bh, bn, kh);
          bl[j] = frag_kc(Bl, bn, kh);
        }
      }
      if constexpr (GEMM3S_DIAG == 3) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
          acc[i][0][0] += (float)(ah[i][0] + al[i][1] + bh[i % FN][2] + bl[i % FN][3]);
        continue;
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
  }

  // epilogue: C/D layout col = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
  if constexpr (GEMM3S_DIAG == 4) {
    // diagnostic: no epilogue stores (every accumulator stays live through
    // a store the compiler cannot prove dead)
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) t += acc[i][j][e];
    if (d.M < 0) ((GLOBAL float*)d.C)[threadIdx.x] = t;
    return;
  }
  // Shuffled through LDS, 32 rows of the wave tile at a time: the MFMA
  // layout gives each lane one column, so direct stores are 2-B (split) or
  // 4-B writes per lane; re-read row-contiguous, every lane stores 8
  // consecutive outputs with 16-B writes (diagnostic build 4 measured the
  // direct-store epilogue at ~35 % of the ResNet-50 chain).  Out-of-range
  // outputs are exactly 0 (zero-padded operands); split images take them
  // into their zero padding, the fp32 output is bounds-checked.
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int CPR = WTN / 8;           // 8-wide chunks per row
  constexpr int RPI = 64 / CPR;          // rows per read instruction
  static_assert(NW * 32 * WTN * 4 <= NSTAGE * STAGE * 2, "epilogue tile must fit the stage LDS");
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // every wave is done with the stage buffers
  float* region = reinterpret_cast<float*>(lds) + w * (32 * WTN);
  const int mw0 = m0 + wr * WTM, nw0 = n0 + wc * WTN;
  // The eigenvalue scaling (S[m][n], or dG[m] for the denominator
  // dG[m] dA[n] + damping) of 16 outputs at a time, loaded together at
  // clamped addresses: 4 memory round trips per wave instead of one per
  // element (loads inside the per-element bounds branch were each waited
  // for alone: 64 dependent round trips per tile in the T2 launch).
  const int kind = d.S != nullptr ? 1 : (d.dg != nullptr ? 2 : 0);
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int cl = j * 32 + (l & 31);
      const int n = nw0 + cl;
      const bool nok = n < d.N;
      const int nc = min(n, d.N - 1);
      float sc[16];
      float dan = 0.f;
      if (kind == 1) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int rl = (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
          const int mc = min(mw0 + i * 32 + rl, d.M - 1);
          sc[e] = ((const GLOBAL float*)d.S)[(int64_t)mc * d.lds + nc];
        }
      } else if (kind == 2) {
        dan = d.da != nullptr ? ((const GLOBAL float*)d.da)[nc] : 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int rl = (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
          sc[e] = ((const GLOBAL float*)d.dg)[min(mw0 + i * 32 + rl, d.M - 1)];
        }
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rl = (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
        const int m = mw0 + i * 32 + rl;
        float v = acc[i][j][e];
        if (!nok || m >= d.M) {
          v = 0.f;
        } else if (kind == 1) {
          v *= sc[e];
        } else if (kind == 2) {
          v = v / (sc[e] * dan + d.damping);
        }
        region[rl * WTN + cl] = v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int t = 0; t < 32 / RPI; ++t) {
      const int rl = t * RPI + l / CPR;
      const int c8 = (l % CPR) * 8;
      typedef float f4 __attribute__((ext_vector_type(4)));
      const f4 x0 = *reinterpret_cast<const f4*>(region + rl * WTN + c8);
      const f4 x1 = *reinterpret_cast<const f4*>(region + rl * WTN + c8 + 4);
      const int m = mw0 + i * 32 + rl;
      const int n = nw0 + c8;
      const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      if constexpr (OUT_SPLIT) {
        // whole chunk, padding included (the image rows / columns are
        // padded to 256 and these values are 0 there)
        typedef unsigned short u8v __attribute__((ext_vector_type(8)));
        u8v hv, lv;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          uint16_t h, lo;
          split1(v[q], h, lo);
          hv[q] = h;
          lv[q] = lo;
        }
        GLOBAL uint16_t* c = (GLOBAL uint16_t*)d.C + (int64_t)m * d.ldc + n;
        *(GLOBAL u8v*)c = hv;
        *(GLOBAL u8v*)(c + d.c_plane) = lv;
      } else {
        if (m < d.M) {
          GLOBAL float* c = (GLOBAL float*)d.C + (int64_t)m * d.ldc + n;
          if (n + 8 <= d.N && (d.ldc & 3) == 0 && (reinterpret_cast<uintptr_t>(d.C) & 15) == 0) {
            *(GLOBAL f4*)c = x0;
            *(GLOBAL f4*)(c + 4) = x1;
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q)
              if (n + q < d.N) c[q] = v[q];
          }
        }
      }
    }
    // the next row group overwrites the region: this wave's reads are done
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
}

// ---- split_pad_multi: fp32 [rows][cols] (+ optional extra column from a
// vector) -> split image planes.  Each thread converts 4 consecutive
// columns of one row.  The padding of the image (columns >= cols (+1), rows
// >= rows) is never written: images are zero-filled once at allocation.
constexpr int SPT = 256;

__device__ __forceinline__ int find_split(const SplitDesc* d, int n, int64_t blk) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].block_start <= blk) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ void __launch_bounds__(SPT)
split_pad_kernel(const SplitDesc* __restrict__ descs, int n) {
  const SplitDesc d = descs[find_split(descs, n, blockIdx.x)];
  const int64_t q = (int64_t)(blockIdx.x - d.block_start) * SPT + threadIdx.x;
  const int total_cols = d.cols + (d.extra != nullptr ? 1 : 0);
  const int qpr = (total_cols + 3) >> 2;  // quads per row
  const int64_t r = q / qpr;
  if (r >= d.rows) return;
  const int c0 = (int)(q - r * qpr) * 4;
  const GLOBAL float* row = (const GLOBAL float*)d.src + r * d.lds;
  float v[4];
  if (d.vec && c0 + 4 <= d.cols) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 x = *(const GLOBAL f4*)(row + c0);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = c0 + e;
      v[e] = c < d.cols ? row[c]
                        : (c == d.cols && d.extra != nullptr ? ((const GLOBAL float*)d.extra)[r] : 0.f);
    }
  }
  uint16_t h[4], lo[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) split1(v[e], h[e], lo[e]);
  GLOBAL uint16_t* dst = (GLOBAL uint16_t*)d.dst + r * d.ldd + c0;
  // the image row stride is a multiple of 128 elements: 8-B aligned quads
  typedef unsigned short u4 __attribute__((ext_vector_type(4)));
  const u4 hh = {h[0], h[1], h[2], h[3]};
  const u4 ll = {lo[0], lo[1], lo[2], lo[3]};
  *(GLOBAL u4*)dst = hh;
  *(GLOBAL u4*)(dst + d.plane) = ll;
}

// Block tile: 2 (256 x 256, 8 waves of 128 x 64, one block per CU) since
// round 5: with the serialised DMA wait and epilogue loads gone, the four
// launches of a step take 1.37 ms (ResNet-50) / 4.62 ms (GPT-NeoX-125M)
// against 1.41 / 5.01 ms with 128 x 128 tiles and 1.69 / 6.21 ms with three
// 128 x 128 stages (profiles/r5/g3s_sweep_epilogue.jsonl).
#ifndef GEMM3S_TILE
#define GEMM3S_TILE 2  // 0: 128x128 (4 waves), 1: 256x128 (8 waves), 2: 256x256 (8 waves), 8: 256x256 (4 waves)
#endif
#ifndef GEMM3S_NSTAGE
#define GEMM3S_NSTAGE 2
#endif
#if GEMM3S_TILE == 0
constexpr int TBM = 128, TBN = 128, TWM = 2, TWN = 2;
#elif GEMM3S_TILE == 1
constexpr int TBM = 256, TBN = 128, TWM = 4, TWN = 2;
#elif GEMM3S_TILE == 3
constexpr int TBM = 128, TBN = 128, TWM = 4, TWN = 2;
#elif GEMM3S_TILE == 4
constexpr int TBM = 256, TBN = 128, TWM = 2, TWN = 2;
#elif GEMM3S_TILE == 5
constexpr int TBM = 128, TBN = 128, TWM = 1, TWN = 2;
#elif GEMM3S_TILE == 6
constexpr int TBM = 128, TBN = 256, TWM = 2, TWN = 2;
#elif GEMM3S_TILE == 7
constexpr int TBM = 128, TBN = 256, TWM = 2, TWN = 4;
#elif GEMM3S_TILE == 8
constexpr int TBM = 256, TBN = 256, TWM = 2, TWN = 2;  // 128 x 128 per wave
#else
constexpr int TBM = 256, TBN = 256, TWM = 2, TWN = 4;
#endif
constexpr int TNS = GEMM3S_NSTAGE;

}  // namespace

// split images are padded to this many rows / columns (every tile config's
// tile edge divides it, so no DMA of an edge tile leaves the image)
int gemm3s_align() { return 256; }
int gemm3s_tile_m() { return TBM; }
int gemm3s_tile_n() { return TBN; }

int gemm3s_grid(int total_tiles) {
  const int per = 8 * CH;
  return ((total_tiles + per - 1) / per) * per;
}

int64_t split_blocks_for(int64_t rows, int64_t total_cols) {
  return ceil_div(rows * ceil_div(total_cols, 4), (int64_t)SPT);
}

void gemm3s_grouped(const Gemm3sDesc* table, int nlayers, int total_tiles, bool a_mc,
                    bool b_mc, bool out_split, hipStream_t s) {
  if (nlayers <= 0 || total_tiles <= 0) return;
  const dim3 grid((unsigned)gemm3s_grid(total_tiles)), block(TWM * TWN * 64);
#define G3S(AM, BM_, OS)                                                                 \
  if (a_mc == AM && b_mc == BM_ && out_split == OS) {                                    \
    gemm3s_kernel<TBM, TBN, TWM, TWN, TNS, AM, BM_, OS><<<grid, block, 0, s>>>(table, nlayers, \
                                                                          total_tiles);  \
    return;                                                                              \
  }
  G3S(false, false, false) G3S(false, false, true) G3S(false, true, false)
  G3S(false, true, true) G3S(true, false, false) G3S(true, false, true)
  G3S(true, true, false) G3S(true, true, true)
#undef G3S
}

void split_pad_multi(const SplitDesc* table, int n, int64_t total_blocks, hipStream_t s) {
  if (n <= 0 || total_blocks <= 0) return;
  split_pad_kernel<<<dim3((unsigned)total_blocks), dim3(SPT), 0, s>>>(table, n);
}

}  // namespace kfac
