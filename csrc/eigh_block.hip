// K-HIP-3 (large-n tier): batched two-sided BLOCK Jacobi eigensolver with a
// warm start from the previous eigenbasis.
//
// Replaces the reference's per-factor torch.linalg.eigh
// (kfac/layers/eigen.py:294-347) for factors above the one-workgroup LDS
// Jacobi tier (eigh_jacobi.hip, n <= 128).  K-FAC factors drift slowly
// between second-order updates, so the host side (eigh_block_host.cpp)
// rotates each factor into the previous eigenbasis, B = Q0^T A Q0 (nearly
// diagonal), and this file diagonalises B by block Jacobi sweeps while
// accumulating V = Q0 * J_1 * J_2 * ...; the eigenvalues are diag(B).
//
// Layout: every matrix is zero-padded to N = k * 32 (k even) so the blocks
// pair up exactly; padded indices stay decoupled (their couplings are and
// remain exactly zero).  One sweep = k - 1 rounds; a round pairs the k
// column blocks (circle method) and for each pair (p, q):
//   bj_pair_solve   one workgroup gathers the 64x64 pair block
//                   [B_pp B_pq; B_qp B_qq] into LDS and diagonalises it with
//                   parallel Jacobi rotations (all 32 disjoint rotations of
//                   an inner round applied in ONE fused LDS pass), giving the
//                   64x64 orthogonal J_P.  Pairs whose off-diagonal norm is
//                   already below the threshold are skipped (J_P = I).
//   bj_apply        B <- J^T B J and V <- V J for all pairs at once: output
//                   groups (P, Q), P <= Q, compute J_P^T B[P,Q] J_Q with fp32
//                   MFMA (v_mfma_f32_32x32x2_f32, exact fp32 products) and
//                   write the mirror; groups (row tile, P) compute V[:,P] J_P.
// The skipped-pair count per sweep is the convergence signal (read by the
// host once per sweep).
#include "common.h"
#include "mfma_tile.h"

namespace kfac {

namespace {

constexpr int BB = 32;          // block edge
constexpr int PB = 2 * BB;      // pair block edge (64)
constexpr int PLD = PB + 1;     // padded LDS row for the pair solve
constexpr int PT = 256;         // threads of the pair solve
constexpr int AT = 256;         // threads of the apply kernel (4 waves)
constexpr int ALD = tile::TILE_LD;  // LDS row of the apply tiles (68 floats)

using tile::v16f;

// circle method over m players (m even): pair k of round r
__device__ __forceinline__ void rr_pair(int m, int r, int k, int& p, int& q) {
  int a, b;
  if (k == 0) {
    a = m - 1;
    b = r;
  } else {
    a = (r + k) % (m - 1);
    b = (r - k + (m - 1)) % (m - 1);
  }
  p = a < b ? a : b;
  q = a < b ? b : a;
}

// global row/col of local index t in pair (p, q)
__device__ __forceinline__ int64_t pair_idx(int p, int q, int t) {
  return t < BB ? (int64_t)p * BB + t : (int64_t)q * BB + (t - BB);
}

struct BJArgs {
  float* B;            // [batch][N][N]
  float* V;            // [batch][N][N]
  float* J;            // [batch][k/2][64][64]
  int* skip;           // [batch][k/2]
  int* active;         // [batch]  non-skipped pairs this sweep
  const float* thr2;   // [batch]  squared absolute off-norm threshold per pair
  int64_t N;
  int k;
  int round;
  int inner_sweeps;
  float noise;         // relative noise floor (x max |diag| of the pair block)
};

// block-wide (sum of x, max of y) over PT threads; every thread gets both
__device__ __forceinline__ void block_sum_max(float x, float y, float* red, float& sum,
                                              float& mx) {
  const int tid = threadIdx.x;
  x = wave_reduce_sum(x);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) y = fmaxf(y, __shfl_xor(y, o, 64));
  if ((tid & 63) == 0) {
    red[2 * (tid >> 6)] = x;
    red[2 * (tid >> 6) + 1] = y;
  }
  __syncthreads();
  sum = 0.f;
  mx = 0.f;
#pragma unroll
  for (int w = 0; w < PT / 64; ++w) {
    sum += red[2 * w];
    mx = fmaxf(mx, red[2 * w + 1]);
  }
  __syncthreads();
}

__global__ void __launch_bounds__(PT)
bj_pair_solve(BJArgs a) {
  __shared__ float S[PB * PLD];
  __shared__ float R[PB * PLD];
  __shared__ float cc[PB];   // cosine of the rotation touching index a
  __shared__ float ss[PB];   // signed sine: y_a = cc[a] x_a + ss[a] x_partner(a)
  __shared__ float red[2 * (PT / 64)];
  const int pair = blockIdx.x, mat = blockIdx.y;
  const int tid = threadIdx.x;
  if (a.active[mat] < 0) return;  // matrix already converged (host flag)
  int p, q;
  rr_pair(a.k, a.round, pair, p, q);
  const float* Bm = a.B + (int64_t)mat * a.N * a.N;

  // gather the 64x64 pair block; R = I
  for (int e = tid; e < PB * PB; e += PT) {
    const int i = e >> 6, j = e & 63;
    S[i * PLD + j] = Bm[pair_idx(p, q, i) * a.N + pair_idx(p, q, j)];
    R[i * PLD + j] = i == j ? 1.f : 0.f;
  }
  __syncthreads();

  auto measure = [&](float& off, float& dmax) {
    float o = 0.f, dm = 0.f;
    for (int e = tid; e < PB * PB; e += PT) {
      const int i = e >> 6, j = e & 63;
      const float v = S[i * PLD + j];
      if (i != j) o += v * v;
      else dm = fmaxf(dm, fabsf(v));
    }
    block_sum_max(o, dm, red, off, dmax);
  };
  float off0, dmax;
  measure(off0, dmax);
  // absolute per-pair threshold, floored at the fp32 noise the apply GEMMs
  // leave next to the block's largest diagonal entry
  const float fl = a.noise * dmax;
  const float thr2 = fmaxf(a.thr2[mat], fl * fl);
  int* skipp = a.skip + (int64_t)mat * (a.k / 2) + pair;
  float* Jm = a.J + ((int64_t)mat * (a.k / 2) + pair) * (PB * PB);
  if (off0 <= thr2) {
    if (tid == 0) *skipp = 1;
    return;
  }
  if (tid == 0) {
    *skipp = 0;
    atomicAdd((int*)(a.active + mat), 1);
  }

  for (int sw = 0; sw < a.inner_sweeps; ++sw) {
    for (int r = 0; r < PB - 1; ++r) {
      // 1) (c, s) of the 32 disjoint rotations of this inner round
      if (tid < PB / 2) {
        int i, j;
        rr_pair(PB, r, tid, i, j);
        float c = 1.f, s = 0.f;
        const float aij = S[i * PLD + j];
        if (aij != 0.f) {
          const float aii = S[i * PLD + i], ajj = S[j * PLD + j];
          const float theta = (ajj - aii) / (2.f * aij);
          const float t = (theta >= 0.f ? 1.f : -1.f) /
                          (fabsf(theta) + sqrtf(theta * theta + 1.f));
          c = rsqrtf(t * t + 1.f);
          s = t * c;
        }
        // row_i' = c row_i - s row_j ; row_j' = s row_i + c row_j (same for
        // columns): zeroes S[i][j]
        cc[i] = c;
        cc[j] = c;
        ss[i] = -s;
        ss[j] = s;
      }
      __syncthreads();
      // 2) S <- G^T S G on 2x2 blocks (one owner per block: in place) and
      //    R <- R G.  Thread t owns column pair kb = t & 31 throughout, so
      //    its column coefficients are read once per round.
      {
        const int kb = tid & 31, ka0 = tid >> 5;
        int b0, b1;
        rr_pair(PB, r, kb, b0, b1);
        const float cb = cc[b0], sb0 = ss[b0], sb1 = ss[b1];
#pragma unroll
        for (int u = 0; u < (PB / 2) * (PB / 2) / PT; ++u) {
          int a0, a1;
          rr_pair(PB, r, ka0 + u * (PT / 32), a0, a1);
          const float ca = cc[a0], sa0 = ss[a0], sa1 = ss[a1];
          const float x00 = S[a0 * PLD + b0], x01 = S[a0 * PLD + b1];
          const float x10 = S[a1 * PLD + b0], x11 = S[a1 * PLD + b1];
          const float y00 = ca * x00 + sa0 * x10, y01 = ca * x01 + sa0 * x11;
          const float y10 = ca * x10 + sa1 * x00, y11 = ca * x11 + sa1 * x01;
          S[a0 * PLD + b0] = cb * y00 + sb0 * y01;
          S[a0 * PLD + b1] = cb * y01 + sb1 * y00;
          S[a1 * PLD + b0] = cb * y10 + sb0 * y11;
          S[a1 * PLD + b1] = cb * y11 + sb1 * y10;
        }
#pragma unroll
        for (int u = 0; u < PB * (PB / 2) / PT; ++u) {
          const int row = ka0 + u * (PT / 32);
          const float v0 = R[row * PLD + b0], v1 = R[row * PLD + b1];
          R[row * PLD + b0] = cb * v0 + sb0 * v1;
          R[row * PLD + b1] = cb * v1 + sb1 * v0;
        }
      }
      __syncthreads();
    }
    float off, dm;
    measure(off, dm);
    if (off <= thr2 * (1.f / 64.f)) break;
  }
  for (int e = tid; e < PB * PB; e += PT) {
    const int i = e >> 6, j = e & 63;
    Jm[e] = R[i * PLD + j];
  }
}

// ---------------------------------------------------------------- apply
// 64x64 tile products: mfma_tile.h (fp32 MFMA, k-major LDS operands)
using tile::mm64;
using tile::store_quad;

__global__ void __launch_bounds__(AT)
bj_apply(BJArgs a, int nb_groups) {
  __shared__ __attribute__((aligned(16))) float X[PB * ALD];   // B tile / V tile
  __shared__ __attribute__((aligned(16))) float JP[PB * ALD];
  __shared__ __attribute__((aligned(16))) float JQ[PB * ALD];
  const int mat = blockIdx.y;
  if (a.active[mat] <= 0) return;  // nothing rotated this round / converged
  const int tid = threadIdx.x;
  const int w = tid >> 6;
  const int wi = w >> 1, wj = w & 1;
  const int np = a.k / 2;
  const int* skip = a.skip + (int64_t)mat * np;
  const float* Jb = a.J + (int64_t)mat * np * (PB * PB);
  const int64_t N = a.N;
  int g = blockIdx.x;
  if (g < nb_groups) {
    // ---- B group (P, Q), P <= Q (upper-triangle enumeration over np)
    int P = 0, rem = g;
    while (rem >= np - P) {
      rem -= np - P;
      ++P;
    }
    const int Q = P + rem;
    const bool sp = skip[P] != 0, sq = skip[Q] != 0;
    if (sp && sq) return;
    int p0, p1, q0, q1;
    rr_pair(a.k, a.round, P, p0, p1);
    rr_pair(a.k, a.round, Q, q0, q1);
    float* Bm = a.B + (int64_t)mat * N * N;
    // load B[P rows][Q cols] and J_P / J_Q (identity when skipped)
    for (int e = tid; e < PB * (PB / 4); e += AT) {
      const int i = e >> 4, c4 = (e & 15) * 4;
      const int64_t gi = pair_idx(p0, p1, i);
      const int64_t gj = pair_idx(q0, q1, c4);  // 4 columns stay in one block
      const float4 v = *reinterpret_cast<const float4*>(Bm + gi * N + gj);
      *reinterpret_cast<float4*>(&X[i * ALD + c4]) = v;
      float4 jp, jq;
      if (sp) jp = make_float4(i == c4, i == c4 + 1, i == c4 + 2, i == c4 + 3);
      else jp = *reinterpret_cast<const float4*>(Jb + (int64_t)P * PB * PB + i * PB + c4);
      if (sq) jq = make_float4(i == c4, i == c4 + 1, i == c4 + 2, i == c4 + 3);
      else jq = *reinterpret_cast<const float4*>(Jb + (int64_t)Q * PB * PB + i * PB + c4);
      *reinterpret_cast<float4*>(&JP[i * ALD + c4]) = jp;
      *reinterpret_cast<float4*>(&JQ[i * ALD + c4]) = jq;
    }
    __syncthreads();
    // T = J_P^T X, stored transposed back into X (after every wave has read X)
    const v16f t = mm64(JP, X, wi, wj);
    __syncthreads();
    store_quad<true>(X, t, wi, wj);
    __syncthreads();
    // O = T J_Q  (A operand = T^T as stored) -> JP (free now)
    const v16f o = mm64(X, JQ, wi, wj);
    __syncthreads();
    store_quad<false>(JP, o, wi, wj);
    __syncthreads();
    // write B[P][Q] and its mirror B[Q][P]; a diagonal group is symmetrised
    for (int e = tid; e < PB * (PB / 4); e += AT) {
      const int i = e >> 4, c4 = (e & 15) * 4;
      float4 v = *reinterpret_cast<const float4*>(&JP[i * ALD + c4]);
      if (P == Q) {
        float* vv = reinterpret_cast<float*>(&v);
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (c4 + u < i) vv[u] = JP[(c4 + u) * ALD + i];
      }
      const int64_t gi = pair_idx(p0, p1, i);
      const int64_t gj = pair_idx(q0, q1, c4);
      *reinterpret_cast<float4*>(Bm + gi * N + gj) = v;
    }
    if (P != Q) {
      // mirror: B[Q rows][P cols] = O^T
      for (int e = tid; e < PB * (PB / 4); e += AT) {
        const int j = e >> 4, c4 = (e & 15) * 4;
        const float4 v = make_float4(JP[c4 * ALD + j], JP[(c4 + 1) * ALD + j],
                                     JP[(c4 + 2) * ALD + j], JP[(c4 + 3) * ALD + j]);
        const int64_t gi = pair_idx(q0, q1, j);
        const int64_t gj = pair_idx(p0, p1, c4);
        *reinterpret_cast<float4*>(Bm + gi * N + gj) = v;
      }
    }
    return;
  }
  // ---- V group (row tile rt of 64 rows, pair P): V[rows][P] <- V[rows][P] J_P
  g -= nb_groups;
  const int P = g % np, rt = g / np;
  if (skip[P]) return;
  int p0, p1;
  rr_pair(a.k, a.round, P, p0, p1);
  float* Vm = a.V + (int64_t)mat * N * N;
  for (int e = tid; e < PB * (PB / 4); e += AT) {
    const int i = e >> 4, c4 = (e & 15) * 4;
    const int64_t gi = (int64_t)rt * PB + i;
    const int64_t gj = pair_idx(p0, p1, c4);
    // V tile stored transposed (X[k][i] = V[i][k]) for the A^T operand
    const float4 v = *reinterpret_cast<const float4*>(Vm + gi * N + gj);
    X[(c4 + 0) * ALD + i] = v.x;
    X[(c4 + 1) * ALD + i] = v.y;
    X[(c4 + 2) * ALD + i] = v.z;
    X[(c4 + 3) * ALD + i] = v.w;
    *reinterpret_cast<float4*>(&JP[i * ALD + c4]) =
        *reinterpret_cast<const float4*>(Jb + (int64_t)P * PB * PB + i * PB + c4);
  }
  __syncthreads();
  const v16f o = mm64(X, JP, wi, wj);
  __syncthreads();
  store_quad<false>(X, o, wi, wj);
  __syncthreads();
  for (int e = tid; e < PB * (PB / 4); e += AT) {
    const int i = e >> 4, c4 = (e & 15) * 4;
    const int64_t gi = (int64_t)rt * PB + i;
    const int64_t gj = pair_idx(p0, p1, c4);
    *reinterpret_cast<float4*>(Vm + gi * N + gj) =
        *reinterpret_cast<const float4*>(&X[i * ALD + c4]);
  }
}

__global__ void bj_sweep_end_kernel(int* active, int batch) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < batch) active[i] = active[i] <= 0 ? -1 : 0;
}

}  // namespace

int bj_block() { return BB; }

// After a sweep: a matrix with no active pair is converged (-1, skipped from
// then on); the others restart their count at 0.
void bj_sweep_end(int* active, int batch, hipStream_t s) {
  bj_sweep_end_kernel<<<dim3((unsigned)((batch + 255) / 256)), dim3(256), 0, s>>>(active, batch);
}

// One round of block Jacobi on a batch of padded [N, N] matrices.
void bj_round(float* B, float* V, float* J, int* skip, int* active, const float* thr2,
              int64_t N, int batch, int round, int inner_sweeps, float noise,
              hipStream_t s) {
  BJArgs a;
  a.B = B;
  a.V = V;
  a.J = J;
  a.skip = skip;
  a.active = active;
  a.thr2 = thr2;
  a.N = N;
  a.k = (int)(N / BB);
  a.round = round;
  a.inner_sweeps = inner_sweeps;
  a.noise = noise;
  const int np = a.k / 2;
  bj_pair_solve<<<dim3((unsigned)np, (unsigned)batch), dim3(PT), 0, s>>>(a);
  const int nb = np * (np + 1) / 2;
  const int nv = (int)(N / PB) * np;
  bj_apply<<<dim3((unsigned)(nb + nv), (unsigned)batch), dim3(AT), 0, s>>>(a, nb);
}

}  // namespace kfac
