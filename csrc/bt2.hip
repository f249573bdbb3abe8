// K-HIP-3, two-stage eigensolver: back-transform of stage 2, X = Q2 Z.
//
// Q2 is the product of the bulge-chasing reflectors H(j, k) (sweep j, task
// k, rows j+1+16k .. +15) in sweep-major order.  Reflectors of 16
// consecutive sweeps g (j = 16g .. 16g+15) at the same task k form one
// compact-WY block B(g, k) = H(16g, k) ... H(16g+15, k) = I - V T V^T on the
// 32 rows starting at s = 16(g+k)+1 (V: 32 x 16, column t = v of sweep 16g+t
// shifted down t rows).  Overlapping reflectors only ever require B(g, k+1)
// before B(g, k) and every block of group g+1 before group g, so
//     X = Q2 Z = prod_{g ascending} [B(g, K) ... B(g, 1) B(g, 0)] Z
// is evaluated by applying the groups from the last to the first, each
// group's blocks in ascending k.  With the step number
//     tau(g, k) = 2 (G - 1 - g) + k
// every block's predecessors have smaller steps and all blocks of one step
// touch disjoint rows (their diagonals q = g + k differ by >= 3), so each
// step is ONE launch over (its blocks) x (column slabs): ~2 n / 16 + n / 16
// launches of independent rank-16 updates instead of n^2 / 32 dependent
// reflector applications (float64 oracle: ops/twostage.py bt2_reference).
//
// bt2_prep_kernel: T of every block (LAPACK larft, forward / columnwise)
// from the stored reflectors, one wave per block.
// bt2_apply_kernel: X[s:s+32, slab] -= V (T (V^T X[s:s+32, slab])).
#include "common.h"

#include <algorithm>

namespace kfac {

namespace {

constexpr int BB = 16;      // band width = reflector length = sweeps per block
constexpr int BR = 2 * BB;  // block rows
constexpr int SLAB = 256;   // columns per workgroup

__device__ __forceinline__ int bt_ntasks(int j, int n) { return 1 + (n - 2 - j) / BB; }

// grid (kmax, G, batch), 64 threads
__global__ void __launch_bounds__(64) bt2_prep_kernel(const float* __restrict__ V2all,
                                                      const float* __restrict__ tau2all,
                                                      int64_t sV2, int n, int kmax, int G,
                                                      float* __restrict__ Tall) {
  const int k = blockIdx.x, g = blockIdx.y, b = blockIdx.z;
  const int j0 = BB * g;
  if (j0 >= n - 2 || k >= bt_ntasks(j0, n)) return;
  const float* V2 = V2all + (int64_t)b * sV2 * BB;
  const float* tau2 = tau2all + (int64_t)b * sV2;
  __shared__ float v[BB][BB + 1];
  __shared__ float tv[BB];
  __shared__ float Gm[BB][BB + 1];
  __shared__ float T[BB][BB + 1];
  const int l = threadIdx.x;
  for (int e = l; e < BB * BB; e += 64) {
    const int t = e / BB, q = e % BB;
    const int j = j0 + t;
    const bool live = j < n - 2 && k < bt_ntasks(j, n);
    v[t][q] = live ? V2[((int64_t)j * kmax + k) * BB + q] : 0.f;
    if (q == 0) tv[t] = live ? tau2[(int64_t)j * kmax + k] : 0.f;
  }
  __syncthreads();
  // Gram of the shifted columns: G[a][t] = sum_q v_a[q] v_t[q - (t - a)]
  for (int e = l; e < BB * BB; e += 64) {
    const int a = e / BB, t = e % BB;
    float s = 0.f;
    if (a < t) {
      const int sh = t - a;
      for (int q = sh; q < BB; ++q) s += v[a][q] * v[t][q - sh];
    }
    Gm[a][t] = s;
    T[a][t] = 0.f;
  }
  __syncthreads();
  for (int t = 0; t < BB; ++t) {
    if (l < t) {
      float acc = 0.f;
      for (int q = l; q < t; ++q) acc += T[l][q] * Gm[q][t];
      T[l][t] = -tv[t] * acc;
    }
    if (l == t) T[t][t] = tv[t];
    __syncthreads();
  }
  float* Tb = Tall + (((int64_t)b * G + g) * kmax + k) * BB * BB;
  for (int e = l; e < BB * BB; e += 64) Tb[e] = T[e / BB][e % BB];
}

// one step: grid (slabs of 256 columns, active groups, batch), 256 threads;
// block (g, k = step - 2 (G-1-g)).  Wave w owns columns c0 + 64 w .. +63
// (four 16-column MFMA tiles); lane l of a tile holds rows
// 16 rt + 4 (l >> 4) + i (rt = 0, 1; i = 0..3) of its column l & 15, and every
// product below sums over a permuted k so that each operand the lane needs
// is already in its own registers: W1 = V^T X (k = row: 8 MFMAs), W2 = T W1
// (k = 4 (l >> 4) + q: 4 MFMAs), X -= V W2 (2 row tiles x 4 MFMAs), all on
// v_mfma_f32_16x16x4_f32 (exact f32).
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) bt2_apply_kernel(
    const float* __restrict__ V2all, int64_t sV2, const float* __restrict__ Tall, int n,
    int kmax, int G, int step, int g_lo, int per, float* __restrict__ Xall, int64_t sX,
    int ldx) {
  const int g = g_lo + (int)blockIdx.y, b = blockIdx.z;
  const int k = step - 2 * (G - 1 - g);
  const int j0 = BB * g;
  if (k < 0 || j0 >= n - 2 || k >= bt_ntasks(j0, n)) return;
  const int s = BB * (g + k) + 1;
  const float* V2 = V2all + (int64_t)b * sV2 * BB;
  const float* Tb = Tall + (((int64_t)b * G + g) * kmax + k) * BB * BB;
  float* X = Xall + (int64_t)b * sX;
  __shared__ float Vs[BR][BB + 1];
  __shared__ float Ts[BB][BB + 1];
  const int tid = threadIdx.x;
  for (int e = tid; e < BR * BB; e += 256) {
    const int rho = e / BB, t = e % BB;
    const int q = rho - t;
    const int j = j0 + t;
    float v = 0.f;
    if (q >= 0 && q < BB && j < n - 2 && k < bt_ntasks(j, n))
      v = V2[((int64_t)j * kmax + k) * BB + q];
    Vs[rho][t] = v;
  }
  Ts[tid / BB][tid % BB] = Tb[tid];
  __syncthreads();
  const int w = tid >> 6, l = tid & 63;
  const int li = l & 15, lh = l >> 4;
  // `per` slabs of 256 columns per workgroup (V, T staged once); a slab's X
  // (4 column tiles x 8 rows per lane) is loaded in one burst before its
  // MFMAs, and the next slab's burst is issued before this slab's MFMAs
  const int sl0 = blockIdx.x * per, sl1 = min((int)(blockIdx.x + 1) * per, (n + 255) / 256);
  float xq[4][8], xn[4][8];
  auto load_slab = [&](int sl, float (&dst)[4][8]) {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int col = sl * 256 + 64 * w + 16 * ct + li;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int row = s + 16 * (q >> 2) + 4 * lh + (q & 3);
        dst[ct][q] = (col < n && row < n) ? X[(int64_t)row * ldx + col] : 0.f;
      }
    }
  };
  if (sl0 < sl1) load_slab(sl0, xq);
  for (int sl = sl0; sl < sl1; ++sl) {
    if (sl + 1 < sl1) load_slab(sl + 1, xn);
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int col = sl * 256 + 64 * w + 16 * ct + li;
      const bool cok = col < n;
      // W1[t][col] = sum_rows V[row][t] X[row][col]
      v4f w1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int rho = 16 * (q >> 2) + 4 * lh + (q & 3);
        w1 = __builtin_amdgcn_mfma_f32_16x16x4f32(Vs[rho][li], xq[ct][q], w1, 0, 0, 0);
      }
      // w1[i] = W1[4 lh + i][col]; W2 = T W1 with k = 4 lh + q
      v4f w2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        w2 = __builtin_amdgcn_mfma_f32_16x16x4f32(Ts[li][4 * lh + q], w1[q], w2, 0, 0, 0);
      // X -= V W2 (row tiles rt = 0, 1; k = 4 lh + q)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        v4f d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 4; ++q)
          d = __builtin_amdgcn_mfma_f32_16x16x4f32(Vs[16 * rt + li][4 * lh + q], w2[q], d, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = s + 16 * rt + 4 * lh + i;
          if (cok && row < n) X[(int64_t)row * ldx + col] = xq[ct][4 * rt + i] - d[i];
        }
      }
    }
    if (sl + 1 < sl1) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int q = 0; q < 8; ++q) xq[ct][q] = xn[ct][q];
    }
  }
}

}  // namespace

int bt2_groups(int n) { return n > 2 ? (int)ceil_div(n - 2, BB) : 0; }

void bt2_prep(const float* V2, const float* tau2, int64_t sV2, int n, int kmax, int batch,
              float* T, hipStream_t stream) {
  const int G = bt2_groups(n);
  if (G == 0 || batch <= 0) return;
  hipLaunchKernelGGL(bt2_prep_kernel, dim3(kmax, G, batch), dim3(64), 0, stream, V2, tau2, sV2,
                     n, kmax, G, T);
}

// X [batch][n][ldx] (row stride ldx, matrix stride sX) <- Q2 X
void bt2_apply(const float* V2, int64_t sV2, const float* T, int n, int kmax, int batch,
               float* X, int64_t sX, int ldx, hipStream_t stream) {
  const int G = bt2_groups(n);
  if (G == 0 || batch <= 0) return;
  const int steps = 2 * (G - 1) + kmax;
  const unsigned slabs = (unsigned)ceil_div(n, SLAB);
  for (int st = 0; st < steps; ++st) {
    // blocks of this step: k = st - 2 (G-1-g) in [0, kmax)
    const int g_lo = std::max(0, G - 1 - st / 2);
    const int g_hi = std::min(G - 1, G - 1 - (st - kmax + 2) / 2);
    if (g_hi < g_lo) continue;
    // ~1024 workgroups per launch: small steps keep one slab per workgroup,
    // large ones give each workgroup several slabs (dispatching thousands of
    // one-slab workgroups per step cost more than their work)
    const int64_t blocks = (int64_t)(g_hi - g_lo + 1) * batch;
    const int per = (int)std::max<int64_t>(1, std::min<int64_t>(slabs, ceil_div(blocks * slabs, 1024)));
    hipLaunchKernelGGL(bt2_apply_kernel, dim3((unsigned)ceil_div(slabs, per), g_hi - g_lo + 1, batch),
                       dim3(256), 0, stream, V2, sV2, T, n, kmax, G, st, g_lo, per, X, sX, ldx);
  }
}

}  // namespace kfac
