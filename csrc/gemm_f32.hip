// Batched fp32 GEMM on the matrix cores, for the GEMM-shaped stages of the
// eigensolver refresh (reference kfac/layers/eigen.py:294-347 runs all of it
// inside torch.linalg.eigh): the blocked back-transform X -= V (T (V^T X))
// (ops/linalg.py apply_q_blocked, csrc/twostage_host.cpp stage-1 BT), the
// divide-and-conquer merges Q_parent = diag(Q1, Q2) W (csrc/tridiag_host.cpp)
// and the triangular inverse of the compact-WY T (gemm_f32_trinv_upper).
//
//   C[b] = alpha * op(A[b]) * op(B[b]) + beta * C[b]        (row-major)
//   op(A) is M x K (A stored [M][lda] or, transposed, [K][lda]),
//   op(B) is K x N (B stored [K][ldb] or, transposed, [N][ldb]).
//
// v_mfma_f32_32x32x2_f32: exact fp32 products with fp32 accumulation (the
// accuracy class of a library sgemm; gfx950 has no TF32), so the refresh
// keeps the float64-parity tests' tolerances.  fp32 MFMA issues at 1/16 of
// the bf16 rate, so the kernel is matrix-core bound once the loads are
// hidden: a 128 x 128 block tile (4 waves in 2 x 2, each 64 x 64 = 2 x 2 MFMA
// 32 x 32 accumulators), k tiles of 32 staged k-major in LDS ([k][m] /
// [k][n], 132-float rows, double buffered: 64 MFMAs per wave cover the next
// tile's global loads), 16-B global loads from a wave-uniform base plus
// 32-bit per-thread offsets (scalar clamped loads at the edges and for
// unaligned operands: any shape, any leading dimension), two blocks per CU.
// 1-D XCD-aware tile order (gemm_f32_kernel).
#include "common.h"

#include <algorithm>
#include <stdexcept>

namespace kfac {

namespace {

constexpr int GT = 128;       // block tile edge
constexpr int GK = 32;        // k per LDS tile
// LDS row strides (floats).  Rows-contiguous operands are stored with 16-B
// writes: 132 (528-B rows, aligned).  k-contiguous operands are transposed
// into LDS by 4-B writes (lane t: k 4 (t & 7) + e, row t >> 3): with 132 the
// 8 k groups of a wave fall on 2 bank groups (PMC: 33 % LDS bank-conflict
// cycles, profiles/r5/pmc/gemmf32.md); 134 = 6 mod 16 spreads them over all
// 64 banks.
constexpr int GLD_RC = GT + 4;
constexpr int GLD_KC = GT + 6;
template <bool RC> constexpr int gld() { return RC ? GLD_RC : GLD_KC; }
constexpr int GTHR = 256;
constexpr int GGM = 8;        // tile rows per group of the tile order

typedef float v16f __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  int64_t lda, ldb, ldc, sA, sB, sC;
  int M, N, K;
  float alpha, beta;
  int ta, tb;
  int splits, kchunk;  // split-K: grid y = batch * splits, partials to ws
  float* ws;
  int tiles_m, tiles_n, per_xcd;
  int vec_a, vec_b;    // 16-B loads allowed (ld % 4 == 0, aligned base)
};

// One operand's k tile: 128 "rows" (m of op(A), n of op(B)) x 32 k, 16
// floats per thread as 4 x 4 consecutive elements of the stored matrix.
//   KC (k contiguous, X[row][ld]): thread t loads k 4 (t & 7) .. +3 of rows
//      (t >> 3) + 32 u          -> 8 threads cover 128 B of a row;
//   RC (rows contiguous, X[k][ld]): thread t loads rows 4 (t & 31) .. +3 at
//      k (t >> 5) + 8 u          -> 32 threads cover 512 B of a k row.
// Offsets are 32-bit from a wave-uniform base that advances by one k tile
// per step (scalar base + vector offset addressing).  Elements outside the
// matrix read as zero; the 16-B path is taken per chunk when the whole chunk
// is inside and the operand is 16-B aligned.
template <bool RC>
struct Tile {
  uint32_t off[4];
  int r0, k0;       // this thread's first row / k inside the tile

  __device__ __forceinline__ void init(int64_t ld) {
    const int t = threadIdx.x;
    if (!RC) {
      k0 = 4 * (t & 7);
      r0 = t >> 3;
#pragma unroll
      for (int u = 0; u < 4; ++u) off[u] = (uint32_t)((r0 + 32 * u) * ld + k0);
    } else {
      r0 = 4 * (t & 31);
      k0 = t >> 5;
#pragma unroll
      for (int u = 0; u < 4; ++u) off[u] = (uint32_t)((k0 + 8 * u) * ld + r0);
    }
  }

  // rows valid below `rlim` (relative to the tile), k below `klim`
  __device__ __forceinline__ void fetch(const float* __restrict__ X, int64_t ld, int rlim, int klim,
                                        bool vec, f4v (&v)[4]) const {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float* p = X + off[u];
      if (!RC) {
        const int r = r0 + 32 * u;
        if (vec && r < rlim && k0 + 4 <= klim) {
          v[u] = *reinterpret_cast<const f4v*>(p);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[u][e] = (r < rlim && k0 + e < klim) ? p[e] : 0.f;
        }
      } else {
        const int k = k0 + 8 * u;
        if (vec && k < klim && r0 + 4 <= rlim) {
          v[u] = *reinterpret_cast<const f4v*>(p);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[u][e] = (k < klim && r0 + e < rlim) ? p[e] : 0.f;
        }
      }
    }
  }

  // LDS image [k][row] (gld<RC>() floats per k row)
  __device__ __forceinline__ void stash(float* S, const f4v (&v)[4]) const {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (!RC) {
#pragma unroll
        for (int e = 0; e < 4; ++e) S[(k0 + e) * GLD_KC + r0 + 32 * u] = v[u][e];
      } else {
        *reinterpret_cast<f4v*>(S + (k0 + 8 * u) * GLD_RC + r0) = v[u];
      }
    }
  }
};

// op(A) rows are m: stored [M][lda] (k contiguous) unless ta; op(B) rows are
// n: stored [N][ldb] (k contiguous) when tb, else [K][ldb] (n contiguous)
template <bool A_RC, bool B_RC>
__global__ void __launch_bounds__(GTHR) gemm_f32_kernel(GemmArgs g) {
  constexpr int LA = gld<A_RC>(), LB = gld<B_RC>();
  __shared__ __attribute__((aligned(16))) float As[2][GK * LA];
  __shared__ __attribute__((aligned(16))) float Bs[2][GK * LB];
  // XCD-aware tile order: the blocks the dispatcher puts on one XCD (every
  // 8th) take a contiguous run of the tile order, and the order walks groups
  // of GGM tile rows column by column, so the blocks resident on an XCD at
  // one time share A row panels and B column panels in that XCD's L2
  const int bid = blockIdx.x;
  const int t = (bid & 7) * g.per_xcd + (bid >> 3);
  if (t >= g.tiles_m * g.tiles_n) return;
  const int per_group = GGM * g.tiles_n;
  const int first_m = (t / per_group) * GGM;
  const int gm = min(g.tiles_m - first_m, GGM);
  const int in_group = t % per_group;
  const int m0 = (first_m + in_group % gm) * GT;
  const int n0 = (in_group / gm) * GT;

  const int64_t b = blockIdx.y / g.splits;
  const int split = blockIdx.y % g.splits;
  // this block's k range [kb, kb + Kc)
  const int kb = split * g.kchunk;
  const int Kc = min(g.K - kb, g.kchunk);
  // tile-origin bases (wave-uniform), advanced by one k tile per step
  const float* A = g.A + b * g.sA + (A_RC ? (int64_t)kb * g.lda + m0 : (int64_t)m0 * g.lda + kb);
  const float* B = g.B + b * g.sB + (B_RC ? (int64_t)kb * g.ldb + n0 : (int64_t)n0 * g.ldb + kb);
  const int64_t stepA = A_RC ? (int64_t)GK * g.lda : GK;
  const int64_t stepB = B_RC ? (int64_t)GK * g.ldb : GK;
  const int rlimA = g.M - m0, rlimB = g.N - n0;
  float* C = g.C + b * g.sC;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const int r = l & 31, h = l >> 5;
  v16f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nk = (Kc + GK - 1) / GK;
  Tile<A_RC> ta;
  Tile<B_RC> tb;
  ta.init(g.lda);
  tb.init(g.ldb);
  const bool va = g.vec_a != 0, vb = g.vec_b != 0;
  f4v ra[4], rb[4];
  ta.fetch(A, g.lda, rlimA, Kc, va, ra);
  tb.fetch(B, g.ldb, rlimB, Kc, vb, rb);
  ta.stash(As[0], ra);
  tb.stash(Bs[0], rb);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      A += stepA;
      B += stepB;
      const int klim = Kc - (kt + 1) * GK;
      ta.fetch(A, g.lda, rlimA, klim, va, ra);
      tb.fetch(B, g.ldb, rlimB, klim, vb, rb);
    }
    const float* as = As[cur];
    const float* bs = Bs[cur];
#pragma unroll
    for (int kk = 0; kk < GK; kk += 2) {
      const float a0 = as[(kk + h) * LA + wm + r];
      const float a1 = as[(kk + h) * LA + wm + 32 + r];
      const float b0 = bs[(kk + h) * LB + wn + r];
      const float b1 = bs[(kk + h) * LB + wn + 32 + r];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (more) {
      ta.stash(As[cur ^ 1], ra);
      tb.stash(Bs[cur ^ 1], rb);
    }
    __syncthreads();
  }
  // C/D layout of v_mfma_f32_32x32x2f32: col = lane & 31,
  // row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + wm + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int col = n0 + wn + 32 * j + r;
        if (row < g.M && col < g.N) {
          if (g.splits > 1) {
            // raw partial [b][split][M][N], summed in split order later
            g.ws[((b * g.splits + split) * g.M + row) * (int64_t)g.N + col] = acc[i][j][e];
            continue;
          }
          float* p = C + (int64_t)row * g.ldc + col;
          const float v = g.alpha * acc[i][j][e];
          *p = g.beta == 0.f ? v : v + g.beta * *p;
        }
      }
}

// C = alpha * sum_s ws[b][s] + beta * C, the splits summed in a fixed order
__global__ void __launch_bounds__(256) gemm_f32_splitk_reduce(GemmArgs g) {
  const int64_t MN = (int64_t)g.M * g.N;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t b = blockIdx.y;
  if (idx >= MN) return;
  const float* src = g.ws + b * g.splits * MN + idx;
  float sum = 0.f;
  for (int s = 0; s < g.splits; ++s) sum += src[s * MN];
  const int row = (int)(idx / g.N), col = (int)(idx % g.N);
  float* p = g.C + b * g.sC + (int64_t)row * g.ldc + col;
  const float v = g.alpha * sum;
  *p = g.beta == 0.f ? v : v + g.beta * *p;
}

}  // namespace

// split-K plan: shapes whose output tiles cannot fill the chip (V V^T of a
// 512-reflector block: 16 tiles over K = 4608) split K into chunks of >= 512
// so the grid reaches ~1024 blocks; workspace batch * splits * M * N floats
// (at most 2^26 floats: fewer splits otherwise)
static int gemm_splits(int M, int N, int K, int batch) {
  const int64_t tiles = ceil_div(M, GT) * ceil_div(N, GT) * (int64_t)batch;
  if (tiles >= 512 || K < 1024) return 1;
  int64_t s = std::min<int64_t>(ceil_div(1024, tiles), K / 512);
  while (s > 1 && s * batch * (int64_t)M * N > (1LL << 26)) --s;
  return (int)std::max<int64_t>(1, s);
}

int64_t gemm_f32_ws_floats(int M, int N, int K, int batch) {
  const int s = gemm_splits(M, N, K, batch);
  return s > 1 ? (int64_t)s * batch * M * N : 0;
}

void gemm_f32_batched(int ta, int tb, int M, int N, int K, float alpha, const float* A,
                      int64_t lda, int64_t sA, const float* B, int64_t ldb, int64_t sB,
                      float beta, float* C, int64_t ldc, int64_t sC, int batch,
                      hipStream_t s, float* ws, int64_t ws_floats) {
  if (M <= 0 || N <= 0 || batch <= 0) return;
  int splits = gemm_splits(M, N, K, batch);
  if (ws == nullptr || ws_floats < (int64_t)splits * batch * M * N) splits = 1;
  const int kchunk = splits > 1 ? (int)(ceil_div(ceil_div(K, splits), GK) * GK) : K;
  splits = splits > 1 ? (int)ceil_div(K, kchunk) : 1;
  const int tm = (int)ceil_div(M, GT), tn = (int)ceil_div(N, GT);
  const int per_xcd = (int)ceil_div((int64_t)tm * tn, 8);
  // 32-bit per-thread offsets inside a tile (Tile::init)
  const int64_t span_a = ta ? (int64_t)GK * lda + GT : (int64_t)GT * lda + GK;
  const int64_t span_b = tb ? (int64_t)GT * ldb + GK : (int64_t)GK * ldb + GT;
  if (span_a >= (int64_t(1) << 31) || span_b >= (int64_t(1) << 31))
    throw std::runtime_error("gemm_f32: operand too large for 32-bit tile offsets");
  auto aligned = [](const float* p, int64_t ld, int64_t stride) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % 4 == 0 && stride % 4 == 0;
  };
  GemmArgs g{A, B, C, lda, ldb, ldc, sA, sB, sC, M, N, K, alpha, beta, ta, tb,
             splits, kchunk > 0 ? kchunk : 1, ws, tm, tn, per_xcd,
             aligned(A, lda, sA) ? 1 : 0, aligned(B, ldb, sB) ? 1 : 0};
  const dim3 grid((unsigned)(8 * per_xcd), (unsigned)(batch * splits));
  const bool arc = ta != 0, brc = tb == 0;
  if (!arc && !brc) hipLaunchKernelGGL((gemm_f32_kernel<false, false>), grid, dim3(GTHR), 0, s, g);
  else if (!arc && brc) hipLaunchKernelGGL((gemm_f32_kernel<false, true>), grid, dim3(GTHR), 0, s, g);
  else if (arc && !brc) hipLaunchKernelGGL((gemm_f32_kernel<true, false>), grid, dim3(GTHR), 0, s, g);
  else hipLaunchKernelGGL((gemm_f32_kernel<true, true>), grid, dim3(GTHR), 0, s, g);
  if (splits > 1) {
    const dim3 rg((unsigned)ceil_div((int64_t)M * N, 256), (unsigned)batch);
    hipLaunchKernelGGL(gemm_f32_splitk_reduce, rg, dim3(256), 0, s, g);
  }
}

}  // namespace kfac

namespace kfac {

namespace {

// in-place inverse of the 64 x 64 upper-triangular diagonal blocks of a
// batch of upper-triangular matrices T ([batch][n][ld]): block (d, b) at
// rows / cols 64 d.  One 64-thread group per block column j: back
// substitution T[i][j] = -(sum_{i < k <= j} U[i][k] T[k][j]) / U[i][i]
// over i = j-1 .. 0, with U staged in LDS.  Entries past n are identity.
constexpr int TB = 64;

__global__ void __launch_bounds__(TB) trinv64_kernel(float* T, int64_t ld, int64_t sT, int n) {
  __shared__ float U[TB][TB + 1];
  const int d = blockIdx.x, j = threadIdx.x;
  float* base = T + (int64_t)blockIdx.y * sT + (int64_t)d * TB * ld + (int64_t)d * TB;
  const int lim = n - d * TB;  // valid rows / cols of this block
  for (int i = 0; i < TB; ++i) {
    float v = (i == j) ? 1.f : 0.f;
    if (i < lim && j < lim) v = base[(int64_t)i * ld + j];
    U[i][j] = v;
  }
  __syncthreads();
  float col[TB];
#pragma unroll
  for (int i = 0; i < TB; ++i) col[i] = 0.f;
  // thread j: column j of U^-1
#pragma unroll
  for (int i = TB - 1; i >= 0; --i) {
    float s = (i == j) ? 1.f : 0.f;
#pragma unroll
    for (int k = i + 1; k < TB; ++k) s -= U[i][k] * col[k];
    col[i] = i <= j ? s / U[i][i] : 0.f;
  }
  for (int i = 0; i < TB; ++i)
    if (i < lim && j < lim) base[(int64_t)i * ld + j] = col[i];
}

}  // namespace

// T <- T^-1 for a batch of n x n upper-triangular matrices (row-major, row
// stride ld, batch stride sT), in place; `work` holds >= batch * n * n / 2
// floats.  64 x 64 diagonal blocks by back substitution, then pairs of
// blocks merged bottom-up: [[T11, X], [0, T22]] with X = -T11 U12 T22
// (two batched GEMMs per merge position).
void trinv_upper_batched(float* T, int64_t ld, int64_t sT, int n, int batch, float* work,
                         hipStream_t s) {
  if (n <= 0 || batch <= 0) return;
  const int nd = (int)ceil_div(n, TB);
  hipLaunchKernelGGL(trinv64_kernel, dim3((unsigned)nd, (unsigned)batch), dim3(TB), 0, s, T, ld,
                     sT, n);
  for (int h = TB; h < n; h *= 2) {
    for (int p = 0; p + h < n; p += 2 * h) {
      const int h2 = (p + 2 * h <= n) ? h : n - p - h;  // second block may be short
      float* t11 = T + (int64_t)p * ld + p;
      float* u12 = T + (int64_t)p * ld + p + h;
      float* t22 = T + (int64_t)(p + h) * ld + p + h;
      // Y = U12 T22 (h x h2), then U12 <- -T11 Y
      gemm_f32_batched(0, 0, h, h2, h2, 1.f, u12, ld, sT, t22, ld, sT, 0.f, work, h2,
                       (int64_t)h * h2, batch, s, nullptr, 0);
      gemm_f32_batched(0, 0, h, h2, h, -1.f, t11, ld, sT, work, h2, (int64_t)h * h2, 0.f, u12,
                       ld, sT, batch, s, nullptr, 0);
    }
  }
}

}  // namespace kfac
