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
// the bf16 rate, so the kernel is matrix-core bound: a 128 x 128 block tile
// (4 waves in 2 x 2, each 64 x 64 = 2 x 2 MFMA 32 x 32 accumulators), k
// tiles of 16 staged k-major in LDS ([k][m] / [k][n], 132-float rows, double
// buffered: the next tile's global loads are in flight during the MFMAs),
// scalar clamped global loads (any shape, any leading dimension, no
// alignment requirement).  Grid (n tiles, m tiles, batch); tiles walk n
// fastest so consecutive blocks share their A row panel in L2.
#include "common.h"

#include <algorithm>

namespace kfac {

namespace {

constexpr int GT = 128;       // block tile edge
constexpr int GK = 16;        // k per LDS tile
constexpr int GLD = GT + 4;   // LDS row (floats)
constexpr int GTHR = 256;

typedef float v16f __attribute__((ext_vector_type(16)));

struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  int64_t lda, ldb, ldc, sA, sB, sC;
  int M, N, K;
  float alpha, beta;
  int ta, tb;
  int splits, kchunk;  // split-K: block z = batch * splits, partials to ws
  float* ws;
};

// Per-thread staging of one operand: 8 elements of every k tile of op(X),
// at fixed (row, k) offsets inside the tile, so the 64-bit addresses are
// formed once per kernel and advanced by a constant per k tile:
//   not transposed (X stored [rows][ld], k contiguous): k = tid & 15,
//     rows (tid >> 4) + 16 u  -> 16 consecutive threads read 64 B of a row;
//   transposed (X stored [K][ld], row contiguous): row = tid & 127,
//     k = (tid >> 7) + 2 u   -> 128 consecutive threads read 512 B.
struct Stager {
  const float* p[8];
  int64_t step;   // pointer advance per k tile
  int rlim[8];    // row valid (not transposed) / k offset in the tile (transposed)
  int kk;         // this thread's k offset in the tile (not transposed)
  bool rok;       // row valid (transposed)
  int trans;

  __device__ __forceinline__ void init(const float* X, int64_t ld, int tr, int rows, int r0) {
    trans = tr;
    const int t = threadIdx.x;
    if (!tr) {
      kk = t & (GK - 1);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = r0 + (t >> 4) + 16 * u;
        rlim[u] = r < rows;
        p[u] = X + (int64_t)(r < rows ? r : 0) * ld + kk;
      }
      step = GK;
    } else {
      const int r = r0 + (t & (GT - 1));
      rok = r < rows;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        rlim[u] = (t >> 7) + 2 * u;
        p[u] = X + (int64_t)rlim[u] * ld + (rok ? r : 0);
      }
      step = (int64_t)GK * ld;
    }
  }

  // load the k tile at k0 (elements past K read as zero)
  __device__ __forceinline__ void fetch(int k0, int K, float (&v)[8]) const {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool ok = trans ? (rok && k0 + rlim[u] < K) : (rlim[u] && k0 + kk < K);
      const float x = ok ? *p[u] : 0.f;
      v[u] = x;
    }
  }

  __device__ __forceinline__ void advance() {
#pragma unroll
    for (int u = 0; u < 8; ++u) p[u] += step;
  }

  __device__ __forceinline__ void stash(float* S, const float (&v)[8]) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (!trans) S[kk * GLD + (t >> 4) + 16 * u] = v[u];
      else S[((t >> 7) + 2 * u) * GLD + (t & (GT - 1))] = v[u];
    }
  }
};

__global__ void __launch_bounds__(GTHR) gemm_f32_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float As[2][GK * GLD];
  __shared__ __attribute__((aligned(16))) float Bs[2][GK * GLD];
  const int n0 = blockIdx.x * GT, m0 = blockIdx.y * GT;
  const int64_t b = blockIdx.z / g.splits;
  const int split = blockIdx.z % g.splits;
  // this block's k range [kb, ke): offset the operands to kb
  const int kb = split * g.kchunk;
  const int Kc = min(g.K - kb, g.kchunk);
  const float* A = g.A + b * g.sA + (g.ta ? (int64_t)kb * g.lda : (int64_t)kb);
  const float* B = g.B + b * g.sB + (g.tb ? (int64_t)kb : (int64_t)kb * g.ldb);
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
  Stager sa, sb;
  sa.init(A, g.lda, g.ta, g.M, m0);
  sb.init(B, g.ldb, !g.tb, g.N, n0);  // op(B)[k][n]: "rows" are n
  float va[8], vb[8];
  sa.fetch(0, Kc, va);
  sb.fetch(0, Kc, vb);
  sa.stash(As[0], va);
  sb.stash(Bs[0], vb);
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < nk;
    if (more) {
      sa.advance();
      sb.advance();
      sa.fetch((t + 1) * GK, Kc, va);
      sb.fetch((t + 1) * GK, Kc, vb);
    }
    const float* as = As[cur];
    const float* bs = Bs[cur];
#pragma unroll
    for (int kk = 0; kk < GK; kk += 2) {
      const float a0 = as[(kk + h) * GLD + wm + r];
      const float a1 = as[(kk + h) * GLD + wm + 32 + r];
      const float b0 = bs[(kk + h) * GLD + wn + r];
      const float b1 = bs[(kk + h) * GLD + wn + 32 + r];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (more) {
      sa.stash(As[cur ^ 1], va);
      sb.stash(Bs[cur ^ 1], vb);
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
  GemmArgs g{A, B, C, lda, ldb, ldc, sA, sB, sC, M, N, K, alpha, beta, ta, tb,
             splits, kchunk > 0 ? kchunk : 1, ws};
  const dim3 grid((unsigned)ceil_div(N, GT), (unsigned)ceil_div(M, GT),
                  (unsigned)(batch * splits));
  hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(GTHR), 0, s, g);
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
