// K-HIP-3 (large-n tier): batched blocked Householder tridiagonalisation of
// symmetric fp32 matrices of MIXED sizes, A = Q T Q^T, Q = H_0 H_1 ... H_{n-2}.
//
// Why: rocSOLVER's syevd reduces one matrix at a time with ~5 dependent
// tiny kernels per column (profiles/rocprof_eigh4608_syevd_stats.csv: 13k
// launches of latrd_* / larfg per 4608 matrix, 55 ms each; the ResNet-50
// factor mix spends ~300 ms of its ~400 ms eigen refresh there, and more
// HIP streams / hardware queues do not overlap the chains:
// profiles/eigh_lanes_hwq_mi355x.jsonl).  Here EVERY large factor a rank owns
// advances one column per launch pair, so the whole mix costs
// 2 * max(n) launches instead of ~5 * sum(n):
//
//   col  (k): finalise column k-1 (normalise its reflector, apply the
//             -tau/2 (w.v) v correction to W), update row k with the
//             panel's V W^T + W V^T, write d[k], and the larfg / W^T x /
//             V^T x partial sums of row k (one workgroup per 256 entries);
//   symv (k): every workgroup re-reduces those partials (beta, tau, v
//             scale, t1 = W^T v, t2 = V^T v), stages v in LDS and computes 8
//             rows of w = tau (A22 v - V t1 - W t2) plus partial w.v;
//   per NB=32 columns: a finalise-only col step and the rank-2NB trailing
//             update A22 -= V W^T + W V^T (64x64 LDS tiles, full square so the
//             trailing matrix stays symmetric and the symv reads whole rows).
//
// Storage is row-major and the math is LAPACK's slatrd / ssytrd with
// uplo = 'L' on the transpose: reflector k (v[k+1] = 1 implicit,
// v[k+2:n] stored) lives in ROW k, which is exactly LAPACK's column-major
// lower layout; the native divide and conquer (csrc/tridiag.hip) and the
// blocked back-transform (ops/linalg.py apply_q_blocked) finish the
// eigensolve (csrc/solver.cpp).  The algorithm is checked step for step on the CPU by
// tools/sytrd_proto.py.  Replaces the reference's torch.linalg.eigh
// (kfac/layers/eigen.py:294-347) for 128 < n <= 8192 (ops/linalg.py).
#include "common.h"
#include "descs.h"

#include <cstdlib>
#include <string>

namespace kfac {

constexpr int SY_NB = 32;                 // panel width
constexpr int SY_T = 256;                 // threads per block
constexpr int SY_P1 = 2 * SY_NB + 4;      // partial stride: xn2, dW[NB], dV[NB]
constexpr int SY_ROWS = 16;               // symv rows per workgroup
constexpr int SY_RPW = SY_ROWS / (SY_T / 64);  // symv rows per wave (4)
// symv column blocks (float4 per lane) in flight per row: a template
// parameter of the symv kernel, chosen by KFAC_SYTRD_SU (4 or 8)
constexpr int SY_MAXN = 8192;             // v staged in LDS (32 KiB)
constexpr int SY_MAXCH = SY_MAXN / SY_T;  // col-step chunks
constexpr int SY_MAXROWBLK = SY_MAXN / SY_ROWS;

int sytrd_nb() { return SY_NB; }
int sytrd_max_n() { return SY_MAXN; }
int sytrd_p1() { return SY_P1; }
int sytrd_maxch() { return SY_MAXCH; }
int sytrd_maxrowblk() { return SY_MAXROWBLK; }

namespace {

// The descriptor's pointers are generic; every access goes through these
// global-address-space views so the compiler emits global_* (not flat_*)
// memory instructions: flat loads also count against lgkmcnt, so each LDS
// wait would drain every outstanding matrix load.
#define GLOBAL __attribute__((address_space(1)))
struct GView {
  GLOBAL float* A;
  GLOBAL float* Wt;
  GLOBAL float* d;
  GLOBAL float* e;
  GLOBAL float* tau;
  GLOBAL float* part1;
  GLOBAL float* part2;
  GLOBAL float* sc;
  GLOBAL float* P;
  int n;
};

__device__ __forceinline__ GView gview(const SytrdDesc& s) {
  return {(GLOBAL float*)s.A,     (GLOBAL float*)s.Wt,    (GLOBAL float*)s.d,
          (GLOBAL float*)s.e,     (GLOBAL float*)s.tau,   (GLOBAL float*)s.part1,
          (GLOBAL float*)s.part2, (GLOBAL float*)s.sc,    (GLOBAL float*)s.P,
          s.n};
}

// Pins every descriptor field in SGPRs at the call site.  Without it the
// compiler loads n first, branches on it, and only then loads the pointers:
// two dependent scalar round trips at the head of every chain kernel.
__device__ __forceinline__ void pin_desc(const GView& D) {
  asm volatile("" ::"s"(D.A), "s"(D.Wt), "s"(D.d), "s"(D.e), "s"(D.tau), "s"(D.part1),
               "s"(D.part2), "s"(D.sc), "s"(D.P), "s"(D.n));
}

// Plain global accesses: every writer and reader of the chain's shared
// data (panel rows, W, the partials) sit in different launches, and the
// kernel boundary orders them.
__device__ __forceinline__ float ldc(const GLOBAL float* p) { return *p; }
__device__ __forceinline__ void stc(GLOBAL float* p, float v) { *p = v; }

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum_uniform(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < SY_T / 64; ++t) s += red[t];
  return s;
}

// col step for column k of panel p (i = k - p).  fin_only: only finalise
// column k-1 (panel end).  grid (chunks, batch).
//
// Latency-bound (a few microseconds of work per column, n of them in a
// chain): every global load of a thread is issued first; the scalars shared
// by the block (the w.v reduction of the previous symv, the panel entries
// of column k) are formed by EVERY wave on its own -- wave reductions and
// lane broadcasts, no LDS round trip -- so the kernel has one block
// barrier, before the final cross-wave sums.
__device__ __forceinline__ void col_body(const GView& D, int bx, int k, int p, int fin_only,
                                         int cnt) {
  const int n = D.n;
  if (k >= n) return;
  const int r0 = k + bx * SY_T;
  if (r0 >= n) return;
  const int i = k - p;
  const int r = r0 + threadIdx.x;
  const bool act = r < n;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __shared__ float wred[SY_T / 64][SY_P1];
  const bool fin = i > 0;  // column k-1 to finalise

  // ---- every global load of this thread first, all in flight together:
  // nothing but the descriptor is loaded before them (cnt, the previous
  // symv's block count, is a kernel argument; rows p + j < n and Wt rows
  // j < NB are always in bounds; values past the panel's current width are
  // masked after the load, never multiplied in)
  float vj[SY_NB], wj[SY_NB];
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < SY_NB; ++j) {
    vj[j] = 0.f;
    wj[j] = 0.f;
  }
  if (act && !fin_only) {
    if (!fin_only) a = ldc(D.A + (int64_t)k * n + r);
#pragma unroll
    for (int j = 0; j < SY_NB; ++j) {
      const int pj = p + j < n ? p + j : n - 1;
      vj[j] = ldc(D.A + (int64_t)pj * n + r);
      wj[j] = ldc(D.Wt + (int64_t)j * n + r);
    }
  }
  float s2 = 0.f;
  if (fin) {
    // partial w.v of column k-1 (one per symv block), summed per wave
    // (G <= SY_MAXROWBLK: a fixed unrolled count, clamped loads, no
    // memory wait per trip)
#pragma unroll
    for (int u = 0; u < SY_MAXROWBLK / 64; ++u) {
      const int t = l + 64 * u;
      const float v = ldc(D.part2 + (t < cnt ? t : cnt - 1));
      s2 += t < cnt ? v : 0.f;
    }
  }
  const float tp = fin ? ldc(D.sc) : 0.f;
  const float sprev = fin ? ldc(D.sc + 1) : 0.f;
  // lane j < i of every wave: W[k, j] and V_j[k] of the panel
  float cw_raw = 0.f, cv_raw = 0.f;
  if (l < i && !fin_only) {
    cw_raw = ldc(D.Wt + (int64_t)l * n + k);
    cv_raw = l == i - 1 ? 1.f : ldc(D.A + (int64_t)(p + l) * n + k);  // V_{i-1}[k] = 1
  }
  float vraw = 0.f, wraw = 0.f;
  if (act && fin) {
    vraw = r == k ? 1.f : ldc(D.A + (int64_t)(k - 1) * n + r);
    wraw = ldc(D.Wt + (int64_t)(i - 1) * n + r);
  }

  const float alpha2 = fin ? -0.5f * tp * wave_sum_uniform(s2) : 0.f;
  // finalised W[k, i-1] gets the -tau/2 (w.v) v correction
  const float cw = l < i ? cw_raw + (l == i - 1 ? alpha2 : 0.f) : 0.f;
  const float cv = l < i ? cv_raw : 0.f;

  float vprev = 0.f, wprev = 0.f;
  if (act && fin) {
    vprev = r == k ? 1.f : vraw * sprev;
    if (r > k) stc(D.A + (int64_t)(k - 1) * n + r, vprev);
    wprev = wraw + alpha2 * vprev;
    // W[k, i-1] is finalised by every block on its own (cw above) and not
    // read again by later col / symv steps: writing it here would race with
    // those reads.  The panel-end trailing update does read it (r = q).
    if (r > k || fin_only) stc(D.Wt + (int64_t)(i - 1) * n + r, wprev);
  }
  if (fin_only) return;

  const int cwi = __builtin_bit_cast(int, cw), cvi = __builtin_bit_cast(int, cv);
#pragma unroll
  for (int j = 0; j < SY_NB; ++j) {
    if (j == i - 1) {
      vj[j] = vprev;
      wj[j] = wprev;
    } else if (j >= i) {
      vj[j] = 0.f;
      wj[j] = 0.f;
    }
    // lane j's panel entries, broadcast (zero for j >= i)
    const float cWj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(cwi, j));
    const float cVj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(cvi, j));
    a -= vj[j] * cWj + wj[j] * cVj;
  }
  if (act) {
    stc(D.A + (int64_t)k * n + r, a);
    if (r == k) stc(D.d + k, a);
  }
  if (k == n - 1) return;  // last diagonal entry: no reflector
  // partial sums over the reflector tail x = a[k+2:n]
  const float x = (act && r >= k + 2) ? a : 0.f;
  float s0 = wave_sum_uniform(x * x);
  if (l == 0) wred[w][0] = s0;
#pragma unroll
  for (int j = 0; j < SY_NB; ++j) {
    // independent reductions; panel columns j >= i are zero and skipped
    // (i is uniform: a scalar branch)
    if (j < i) {
      const float sw = wave_sum_uniform(wj[j] * x);
      const float sv = wave_sum_uniform(vj[j] * x);
      if (l == 0) {
        wred[w][1 + j] = sw;
        wred[w][1 + SY_NB + j] = sv;
      }
    }
  }
  __syncthreads();
  const int nval = 1 + 2 * SY_NB;
  for (int t = threadIdx.x; t < nval; t += SY_T) {
    const int j = (t - 1) % SY_NB;
    if (t > 0 && j >= i) continue;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < SY_T / 64; ++q) s += wred[q][t];
    stc(D.part1 + (int64_t)bx * SY_P1 + t, s);
  }
}

__global__ void __launch_bounds__(SY_T) sytrd_col_kernel(
    const SytrdDesc* __restrict__ descs, int k, int p, int fin_only, int cnt) {
  const GView D = gview(descs[blockIdx.y]);
  pin_desc(D);
  col_body(D, blockIdx.x, k, p, fin_only, cnt);
}

// symv step for column k (k <= n-2).  grid (G, batch), G = sytrd_symv_blocks().
//
// Rows are dealt to WAVES, not blocks: global wave g = 4 b + w of the
// member's G blocks takes rows k+1+g, k+1+g+4G, ... two at a time, so every
// wave of a launch streams the same number of rows (+-1) whatever n - k is
// -- with 16-row blocks, 288 blocks for one 4608 factor at column 0 put two
// blocks on 32 of the 256 CUs.  The matrix stream does not depend on the
// reflector scalars (v is staged raw; the scale is applied to each row's
// sum), so each wave's first two rows are loaded before the prologue, and
// after ONE block barrier (staged v and partials visible) each wave forms
// the scalars and its panel correction terms on its own.  Every block
// writes its partial w.v (0 without rows) to part2[b]; the next col step
// gets G as an argument.
template <int SY_SU>
__device__ __forceinline__ void symv_body(const GView& D, int bx, int G, int k, int p) {
  const int n = D.n;
  if (k >= n - 1) return;  // this member is done (its col steps stop too)
  const int i = k - p;
  __shared__ __attribute__((aligned(16))) float sv[SY_MAXN];
  __shared__ float ptmp[SY_MAXCH * SY_P1];
  __shared__ float red[SY_T / 64];

  typedef float f4 __attribute__((ext_vector_type(4)));
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int W = 4 * G;                                  // waves of this member
  const int r_first = k + 1 + bx * 4 + wv;  // this wave's first row
  const int base = (k + 1) & ~3;
  const int span = n - base;
  const bool vec = (n & 3) == 0;  // rows 16-B aligned
  const int nq = span >> 2;
  // ---- (1) this wave's first two rows, first SY_SU column blocks
  f4 a4[2][SY_SU];
  const bool first = vec && r_first < n;
  if (first) {
    const int rb = r_first + W < n ? r_first + W : r_first;
    const GLOBAL float* p0 = D.A + (int64_t)r_first * n + base;
    const GLOBAL float* p1 = D.A + (int64_t)rb * n + base;
#pragma unroll
    for (int u = 0; u < SY_SU; ++u) {
      const int q = l + 64 * u < nq ? l + 64 * u : 0;
      a4[0][u] = *(const GLOBAL f4*)(p0 + 4 * q);
      a4[1][u] = *(const GLOBAL f4*)(p1 + 4 * q);
    }
  }
  // ---- (2) prologue: the col step's partials of column k, the raw
  // reflector row, this lane's panel entry of column k+1, the pivot
  // (fixed-count unrolled loads: a plain strided loop is vectorised 8 wide
  // with a full memory wait per trip -- 3-4 dependent round trips at n=4608)
  // lane l < i: W[k+1, l]; lane 32 <= l < 32 + i: V_{l-32}[k+1]
  float wa = 0.f;
  if (l < i) wa = ldc(D.Wt + (int64_t)l * n + k + 1);
  else if (l >= 32 && l - 32 < i) wa = ldc(D.A + (int64_t)(p + l - 32) * n + k + 1);
  const float alpha = ldc(D.A + (int64_t)k * n + k + 1);
  const int nch = (int)ceil_div(n - k, SY_T);
  const int np1 = nch * SY_P1;
  constexpr int PT = (SY_MAXCH * SY_P1 + SY_T - 1) / SY_T;
  float pst[PT];
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    const int t = threadIdx.x + SY_T * u;
    pst[u] = ldc(D.part1 + (t < np1 ? t : np1 - 1));  // clamped: no branch per load
  }
  const GLOBAL float* arow = D.A + (int64_t)k * n;
  constexpr int VT = SY_MAXN / SY_T;
  float vst[VT];
#pragma unroll
  for (int u = 0; u < VT; ++u) {
    const int c = threadIdx.x + SY_T * u;
    const float v = ldc(arow + (c < span ? base + c : n - 1));
    vst[u] = base + c > k + 1 ? v : 0.f;
  }
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    const int t = threadIdx.x + SY_T * u;
    if (t < np1) ptmp[t] = pst[u];
  }
#pragma unroll
  for (int u = 0; u < VT; ++u) {
    const int c = threadIdx.x + SY_T * u;
    if (c < span) sv[c] = vst[u];
  }
  __syncthreads();

  // ---- (3) reflector scalars, per wave: ||x||^2 and this lane's
  // V^T x / W^T x partial totals (lane l needs entry 1 + l either way)
  float xn2 = 0.f, xl = 0.f;
  for (int c = 0; c < nch; ++c) {
    xn2 += ptmp[c * SY_P1];
    xl += ptmp[c * SY_P1 + 1 + l];
  }
  float tau_k, beta, scale;
  if (xn2 == 0.f) {
    tau_k = 0.f;
    beta = alpha;
    scale = 0.f;
  } else {
    beta = -copysignf(sqrtf(alpha * alpha + xn2), alpha);
    tau_k = (beta - alpha) / beta;
    scale = 1.f / (alpha - beta);
  }
  if (bx == 0 && threadIdx.x == 0) {
    stc(D.e + k, beta);
    stc(D.tau + k, tau_k);
    stc(D.sc, tau_k);
    stc(D.sc + 1, scale);
  }
  // t1 = W^T v (lanes < i), t2 = V^T v (lanes 32 .. 32 + i)
  const bool tlive = l < i || (l >= 32 && l - 32 < i);
  const float tl = tlive ? wa + scale * xl : 0.f;

  // ---- (4) rows: y_raw = A22 a_raw, then w = tau (A22 v - V t1 - W t2)
  float pd = 0.f;
  bool pre = first;
  for (int r0 = r_first; r0 < n; r0 += 2 * W) {
    const int r1 = r0 + W;
    const bool two = r1 < n;
    const int r1c = two ? r1 : r0;
    // this pair's panel entries (lanes < i: V rows, 32.. : W rows) and
    // column k+1 entries
    float pv0 = 0.f, pv1 = 0.f;
    if (l < i) {
      pv0 = ldc(D.A + (int64_t)(p + l) * n + r0);
      pv1 = ldc(D.A + (int64_t)(p + l) * n + r1c);
    } else if (l >= 32 && l - 32 < i) {
      pv0 = ldc(D.Wt + (int64_t)(l - 32) * n + r0);
      pv1 = ldc(D.Wt + (int64_t)(l - 32) * n + r1c);
    }
    const float pk0 = D.A[(int64_t)r0 * n + k + 1];
    const float pk1 = D.A[(int64_t)r1c * n + k + 1];
    float acc0 = 0.f, acc1 = 0.f;
    if (vec) {
      const GLOBAL float* p0 = D.A + (int64_t)r0 * n + base;
      const GLOBAL float* p1 = D.A + (int64_t)r1c * n + base;
      int q = l;
      for (; q < nq; q += 64 * SY_SU) {
        if (!pre) {
#pragma unroll
          for (int u = 0; u < SY_SU; ++u) {
            const int qq = q + 64 * u < nq ? q + 64 * u : 0;
            a4[0][u] = *(const GLOBAL f4*)(p0 + 4 * qq);
            a4[1][u] = *(const GLOBAL f4*)(p1 + 4 * qq);
          }
        }
        pre = false;
#pragma unroll
        for (int u = 0; u < SY_SU; ++u) {
          if (q + 64 * u < nq) {
            const f4 vv = *reinterpret_cast<const f4*>(sv + 4 * (q + 64 * u));
            acc0 += (a4[0][u].x * vv.x + a4[0][u].y * vv.y) +
                    (a4[0][u].z * vv.z + a4[0][u].w * vv.w);
            acc1 += (a4[1][u].x * vv.x + a4[1][u].y * vv.y) +
                    (a4[1][u].z * vv.z + a4[1][u].w * vv.w);
          }
        }
      }
      pre = false;  // (lanes past nq never entered the loop)
    } else {
      for (int c = l; c < span; c += 64) {
        const float vc = sv[c];
        acc0 += D.A[(int64_t)r0 * n + base + c] * vc;
        acc1 += D.A[(int64_t)r1c * n + base + c] * vc;
      }
    }
    // y = A22 v with v = [1, scale * a]
    const float y0 = pk0 + scale * wave_sum_uniform(acc0);
    const float c0 = wave_sum_uniform(pv0 * tl);
    const float w0 = tau_k * (y0 - c0);
    const float y1 = pk1 + scale * wave_sum_uniform(acc1);
    const float c1 = wave_sum_uniform(pv1 * tl);
    const float w1 = tau_k * (y1 - c1);
    if (l == 0) {
      stc(D.Wt + (int64_t)i * n + r0, w0);
      pd += w0 * (r0 == k + 1 ? 1.f : scale * sv[r0 - base]);
      if (two) {
        stc(D.Wt + (int64_t)i * n + r1, w1);
        pd += w1 * (r1 == k + 1 ? 1.f : scale * sv[r1 - base]);
      }
    }
  }
  pd = block_sum(pd, red);
  if (threadIdx.x == 0) stc(D.part2 + bx, pd);
}

template <int SY_SU>
__global__ void __launch_bounds__(SY_T) sytrd_symv_kernel(
    const SytrdDesc* __restrict__ descs, int k, int p) {
  const GView D = gview(descs[blockIdx.y]);
  pin_desc(D);
  symv_body<SY_SU>(D, blockIdx.x, gridDim.x, k, p);
}

// trailing update A[q:,q:] -= V W^T + W V^T for the panel [p, q).
// grid (col tiles, row tiles, batch), 64x64 tiles, 16x16 threads x 4x4.
__global__ void __launch_bounds__(SY_T) sytrd_syr2k_kernel(
    const SytrdDesc* __restrict__ descs, int q, int p) {
  const GView D = gview(descs[blockIdx.z]);
  pin_desc(D);
  const int n = D.n;
  if (q >= n) return;
  const int r0 = q + blockIdx.y * 64, c0 = q + blockIdx.x * 64;
  if (r0 >= n || c0 >= n) return;
  const int mw = q - p;
  __shared__ float Vr[SY_NB][64], Wr[SY_NB][64], Vc[SY_NB][64], Wc[SY_NB][64];
  // every panel load of the thread first, at clamped in-bounds addresses
  // (masked when stored): one memory round trip.  (Guarded loads inside
  // the staging loop were waited for one iteration at a time; with the
  // per-element read-modify-write below that made this a ~36 us kernel of
  // dependent round trips on the chain's critical path, 4 FMAs of work per
  // load.)
  constexpr int ST = SY_NB * 64 / SY_T;  // staging trips per thread
  float vr[ST], wr[ST], vc[ST], wc[ST];
#pragma unroll
  for (int u = 0; u < ST; ++u) {
    const int t = threadIdx.x + u * SY_T;
    const int j = t >> 6, x = t & 63;
    const int jj = j < mw ? j : 0;
    const int r = min(r0 + x, n - 1), c = min(c0 + x, n - 1);
    vr[u] = D.A[(int64_t)(p + jj) * n + r];
    wr[u] = D.Wt[(int64_t)jj * n + r];
    vc[u] = D.A[(int64_t)(p + jj) * n + c];
    wc[u] = D.Wt[(int64_t)jj * n + c];
  }
#pragma unroll
  for (int u = 0; u < ST; ++u) {
    const int t = threadIdx.x + u * SY_T;
    const int j = t >> 6, x = t & 63;
    const int r = r0 + x, c = c0 + x;
    const bool live = j < mw;
    Vr[j][x] = (live && r < n) ? (r == p + j + 1 ? 1.f : vr[u]) : 0.f;
    Wr[j][x] = (live && r < n) ? wr[u] : 0.f;
    Vc[j][x] = (live && c < n) ? (c == p + j + 1 ? 1.f : vc[u]) : 0.f;
    Wc[j][x] = (live && c < n) ? wc[u] : 0.f;
  }
  __syncthreads();
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float acc[4][4] = {};
  for (int j = 0; j < mw; ++j) {
    float vr[4], wr[4], vc[4], wc[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      vr[a] = Vr[j][ty * 4 + a];
      wr[a] = Wr[j][ty * 4 + a];
      vc[a] = Vc[j][tx + 16 * a];
      wc[a] = Wc[j][tx + 16 * a];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] += vr[a] * wc[b] + wr[a] * vc[b];
  }
  // read-modify-write of the 4 x 4 outputs: the old values loaded together
  float old[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
      old[a][b] = D.A[(int64_t)min(r0 + ty * 4 + a, n - 1) * n + min(c0 + tx + 16 * b, n - 1)];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int r = r0 + ty * 4 + a;
    if (r >= n) continue;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int c = c0 + tx + 16 * b;
      if (c < n) D.A[(int64_t)r * n + c] = old[a][b] - acc[a][b];
    }
  }
}

}  // namespace

// symv blocks per member for `rows` rows of the largest member: the whole
// launch (blocks x batch) is sized to `waves` waves, with every wave
// streaming the same number of rows.  Default 6144 = twice the chip's
// resident waves (3 blocks of 4 waves per CU): on the ResNet-50 mix, whose
// three chains run concurrently, 215 ms vs 238 ms with one chip's worth and
// 383-474 ms with smaller budgets for the smaller chains
// (profiles/r4_eigh/mix_w*.jsonl).  KFAC_SYTRD_WAVES overrides per chain.
int sytrd_symv_blocks(int rows, int batch, int waves) {
  if (rows <= 0) return 1;
  if (waves <= 0) waves = 6 * 256 * 4;
  const int per = (int)ceil_div((int64_t)rows * batch, (int64_t)waves);  // rows per wave
  int g = (int)ceil_div((int64_t)rows, (int64_t)4 * per);
  if (g > SY_MAXROWBLK) g = SY_MAXROWBLK;
  return g < 1 ? 1 : g;
}

// Host driver: descs is a device table of `batch` descriptors, ns the host
// copy of their sizes.  Issues 2 launches per column of the largest matrix
// plus 2 per panel, all on `stream`, no host sync.  (A persistent one-launch-
// per-panel form with device-wide barriers and a lower-triangle tile symv
// were measured slower -- 4608: 194 / 142 ms vs 103 ms, profiles/r5/
// eigh_variants/ -- and removed in round 6.)
void sytrd_batched_range(const SytrdDesc* descs_dev, const int* ns, int batch,
                         int k_begin, int k_end, hipStream_t stream, int waves) {
  int maxn = 0;
  for (int b = 0; b < batch; ++b) maxn = ns[b] > maxn ? ns[b] : maxn;
  if (maxn <= 0) return;
  if (k_end > maxn) k_end = maxn;
  static const int su = [] {
    const char* e = getenv("KFAC_SYTRD_SU");
    return e && atoi(e) == 8 ? 8 : 4;
  }();
  // segments start on panel boundaries: panel [p, p+NB) is issued whole
  for (int p = k_begin; p < k_end; p += SY_NB) {
    const int q = (p + SY_NB < maxn) ? p + SY_NB : maxn;
    for (int k = p; k < q; ++k) {
      const int rem = maxn - k;
      // the previous column's symv had maxn - k rows in the largest member
      hipLaunchKernelGGL(sytrd_col_kernel, dim3((unsigned)ceil_div(rem, SY_T), batch),
                         dim3(SY_T), 0, stream, descs_dev, k, p, 0,
                         sytrd_symv_blocks(maxn - k, batch, waves));
      if (k < maxn - 1) {
        const dim3 grid((unsigned)sytrd_symv_blocks(rem - 1, batch, waves), batch);
        if (su == 8)
          hipLaunchKernelGGL(sytrd_symv_kernel<8>, grid, dim3(SY_T), 0, stream, descs_dev, k, p);
        else
          hipLaunchKernelGGL(sytrd_symv_kernel<4>, grid, dim3(SY_T), 0, stream, descs_dev, k, p);
      }
    }
    if (q < maxn) {
      const int rem = maxn - q;
      hipLaunchKernelGGL(sytrd_col_kernel, dim3((unsigned)ceil_div(rem, SY_T), batch),
                         dim3(SY_T), 0, stream, descs_dev, q, p, 1,
                         sytrd_symv_blocks(maxn - q, batch, waves));
      const unsigned tiles = (unsigned)ceil_div(rem, 64);
      hipLaunchKernelGGL(sytrd_syr2k_kernel, dim3(tiles, tiles, batch), dim3(SY_T), 0,
                         stream, descs_dev, q, p);
    }
  }
}

// Whole reduction in one call: 2 launches per column of the largest matrix
// plus 2 per panel.  A matrix of size n is complete once the panels up to n
// have been issued (later launches return early for it), which lets the
// caller split the chain into segments and finish small matrices early.
void sytrd_batched(const SytrdDesc* descs_dev, const int* ns, int batch,
                   hipStream_t stream) {
  sytrd_batched_range(descs_dev, ns, batch, 0, 1 << 30, stream, 0);
}

}  // namespace kfac
