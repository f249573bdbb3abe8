// K-HIP-3, two-stage eigensolver, stage 1: dense symmetric -> band (width 16).
//
// A = Q1 B Q1^T with B banded (|i - j| <= 16).  Panel p (columns p..p+15,
// rows p+16..n-1, m = n - p - 16 rows) is factored P = Q_p R by Householder
// QR; the trailing matrix is then updated two-sidedly,
//   A22 <- Q_p^T A22 Q_p,  Q_p = I - V T V^T,
// with level-3 operations only (Y = A22 V T, W = Y - 1/2 V sym(T^T V^T Y),
// A22 -= V W^T + W V^T: sb_symm / sb_sred / sb_upd below, three launches per
// panel working in place on the leading-dimension-ld storage).  The one-stage Householder tridiagonalisation
// (csrc/sytrd.hip) streams the whole trailing matrix once per COLUMN
// (a matrix-vector product, HBM-bound); here it is streamed twice per 16
// columns by GEMMs.  Replaces the reference's torch.linalg.eigh
// (kfac/layers/eigen.py:294-347); float64 oracle:
// distributed_kfac_pytorch_amd/ops/twostage.py.
//
// sb_qr_kernel: one 1024-thread workgroup per matrix holds its whole panel in
// registers (RPT rows x 16 columns per thread) and runs the 16 Householder
// steps with two block reductions each; the dot products of the new
// reflector with the previous ones come out of the same reduction as the
// trailing-column products, so the compact-WY factor T (LAPACK larft,
// forward / columnwise) costs nothing extra.  Outputs:
//   A lower panel  <- R (upper triangular 16 x 16: the band) and the
//                     reflectors below it (column p+a holds v_a, v_a[p+16+a] = 1
//                     implicit: the layout the blocked back-transform reads);
//   V [m][16], U = V T [m][16], T [16][16], tau1[p+a].
#include "common.h"

namespace kfac {

constexpr int TS_B = 16;         // band width = panel width
constexpr int QR_T = 1024;       // threads of the panel QR
constexpr int QR_W = QR_T / 64;  // waves
constexpr int QR_RPT_MAX = 5;    // rows per thread -> m <= 5120

int twostage_band() { return TS_B; }
int twostage_max_n() { return QR_RPT_MAX * QR_T + TS_B; }

namespace {

// sum over the 16 lanes of each DPP row, left in every lane of the row
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_mov<0xb1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_mov<0x4e>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v;
}

// block-wide sums of 16 per-thread values; every thread receives the totals.
// Per value a 4-step DPP row sum; lane 0 of each 16-lane row deposits its 16
// row sums (red: [QR_T / 16][16]); wave q then folds the 64 row sums of value
// q with one LDS read per lane and a wave reduction (a serial loop over the
// 64 partials cost ~1.5 us per column).
__device__ __forceinline__ void block_sum16(float (&v)[TS_B], float* red, float* tot) {
  const int row = threadIdx.x >> 4, l16 = threadIdx.x & 15;
#pragma unroll
  for (int c = 0; c < TS_B; ++c) {
    const float s = row_sum16(v[c]);
    if (l16 == 0) red[row * TS_B + c] = s;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  static_assert(QR_W == TS_B && QR_T / 16 == 64, "one wave per value, 64 row sums each");
  const float t = wave_sum_uniform(red[l * TS_B + w]);
  if (l == 0) tot[w] = t;
  __syncthreads();
#pragma unroll
  for (int c = 0; c < TS_B; ++c) v[c] = tot[c];
}

__device__ __forceinline__ float block_sum1(float v, float* red, float* tot) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const float s = wave_sum_uniform(v);
  if (l == 0) red[w] = s;
  __syncthreads();
  if (w == 0) {
    const float t = wave_sum_uniform(l < QR_W ? red[l] : 0.f);
    if (l == 0) tot[0] = t;
  }
  __syncthreads();
  return tot[0];
}

template <int RPT>
__global__ void __launch_bounds__(QR_T) sb_qr_kernel(
    float* __restrict__ A, int64_t sA, int ld, int n, int p, float* __restrict__ Vw,
    float* __restrict__ Uw, int64_t sVU, float* __restrict__ tau1, int64_t sTau,
    float* __restrict__ Tw) {
  const int b = blockIdx.x;
  float* Ab = A + (int64_t)b * sA;
  const int m = n - p - TS_B;
  const int tid = threadIdx.x;
  __shared__ float red[(QR_T / 16) * TS_B];
  __shared__ float tot[TS_B];
  __shared__ float Ts[TS_B][TS_B + 1];
  __shared__ float alpha_s;
  // rows s < RR in registers, the rest in LDS ([s - RR][column][thread]:
  // consecutive threads, consecutive words) -- no scratch spills at RPT 4, 5
  constexpr int RR = RPT == 5 ? 3 : (RPT < 2 ? RPT : 2);  // LDS holds <= 2 rows (128 KiB)
  constexpr int RL = RPT - RR;
  __shared__ float PL[(RL > 0 ? RL : 1) * TS_B * QR_T];
  float PR[RR][TS_B];
#define PX(s_, c_) (*((s_) < RR ? &PR[(s_) < RR ? (s_) : 0][c_] : &PL[(((s_) >= RR ? (s_) - RR : 0) * TS_B + (c_)) * QR_T + tid]))
#pragma unroll
  for (int s = 0; s < RPT; ++s) {
    const int i = tid + QR_T * s;
    if (i < m) {
      const float4* row = reinterpret_cast<const float4*>(Ab + (int64_t)(p + TS_B + i) * ld + p);
#pragma unroll
      for (int q = 0; q < TS_B / 4; ++q) {
        const float4 x = row[q];
        PX(s, 4 * q) = x.x;
        PX(s, 4 * q + 1) = x.y;
        PX(s, 4 * q + 2) = x.z;
        PX(s, 4 * q + 3) = x.w;
      }
    } else {
#pragma unroll
      for (int c = 0; c < TS_B; ++c) PX(s, c) = 0.f;
    }
  }
  if (tid < TS_B * (TS_B + 1)) (&Ts[0][0])[tid] = 0.f;
  const int bb = m < TS_B ? m : TS_B;

#pragma unroll
  for (int t = 0; t < TS_B; ++t) {
    if (t < bb) {
      // ---- Householder vector of column t (rows t..m-1)
      float part = 0.f;
#pragma unroll
      for (int s = 0; s < RPT; ++s) {
        const int i = tid + QR_T * s;
        if (i > t && i < m) part += PX(s, t) * PX(s, t);
      }
      if (tid == t) alpha_s = PX(0, t);
      const float xn2 = block_sum1(part, red, tot);
      const float alpha = alpha_s;
      float tau, beta, scale;
      if (xn2 == 0.f) {
        tau = 0.f;
        beta = alpha;
        scale = 0.f;
      } else {
        beta = -copysignf(sqrtf(alpha * alpha + xn2), alpha);
        tau = (beta - alpha) / beta;
        scale = 1.f / (alpha - beta);
      }
      float vv[RPT];
#pragma unroll
      for (int s = 0; s < RPT; ++s) {
        const int i = tid + QR_T * s;
        vv[s] = i == t ? 1.f : ((i > t && i < m) ? PX(s, t) * scale : 0.f);
      }
      // ---- u_c = v^T P[:, c]: trailing columns (c > t) for the update,
      // earlier columns (c < t: the stored reflectors) for T
      float u[TS_B];
#pragma unroll
      for (int c = 0; c < TS_B; ++c) {
        float a = 0.f;
        if (c != t) {
#pragma unroll
          for (int s = 0; s < RPT; ++s) a += vv[s] * PX(s, c);
        }
        u[c] = a;
      }
      block_sum16(u, red, tot);
#pragma unroll
      for (int c = t + 1; c < TS_B; ++c) {
        const float f = tau * u[c];
#pragma unroll
        for (int s = 0; s < RPT; ++s) PX(s, c) -= f * vv[s];
      }
#pragma unroll
      for (int s = 0; s < RPT; ++s) {
        const int i = tid + QR_T * s;
        if (i == t) PX(s, t) = beta;
        else if (i > t) PX(s, t) = vv[s];
      }
      // ---- T column t: T[a][t] = -tau sum_{q=a}^{t-1} T[a][q] u[q]
      if (tid < t) {
        float acc = 0.f;
        for (int q = tid; q < t; ++q) acc += Ts[tid][q] * u[q];
        Ts[tid][t] = -tau * acc;
      }
      if (tid == t) {
        Ts[t][t] = tau;
        tau1[(int64_t)b * sTau + p + t] = tau;
      }
    } else if (tid == 0) {
      tau1[(int64_t)b * sTau + p + t] = 0.f;
    }
  }
  __syncthreads();

  // ---- outputs
  float* Vb = Vw + (int64_t)b * sVU;
  float* Ub = Uw + (int64_t)b * sVU;
#pragma unroll
  for (int s = 0; s < RPT; ++s) {
    const int i = tid + QR_T * s;
    if (i >= m) continue;
    float v[TS_B];
#pragma unroll
    for (int a = 0; a < TS_B; ++a) v[a] = i > a ? PX(s, a) : (i == a ? 1.f : 0.f);
    float4* vrow = reinterpret_cast<float4*>(Vb + (int64_t)i * TS_B);
    float4* urow = reinterpret_cast<float4*>(Ub + (int64_t)i * TS_B);
#pragma unroll
    for (int q = 0; q < TS_B / 4; ++q) {
      float uq[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 4 * q + e;
        float acc = 0.f;
#pragma unroll
        for (int a = 0; a <= c; ++a) acc += v[a] * Ts[a][c];
        uq[e] = acc;
      }
      vrow[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
      urow[q] = make_float4(uq[0], uq[1], uq[2], uq[3]);
    }
    // lower panel <- the factored panel: R on and above the diagonal (the
    // band), reflector v_a below it in column p+a (v_a[p+16+a] = 1 implicit;
    // the blocked back-transform reads it there).  Nothing here is inside the
    // trailing matrix, so the next panel's QR may overlap this panel's update.
    float4* arow = reinterpret_cast<float4*>(Ab + (int64_t)(p + TS_B + i) * ld + p);
#pragma unroll
    for (int q = 0; q < TS_B / 4; ++q)
      arow[q] = make_float4(PX(s, 4 * q), PX(s, 4 * q + 1), PX(s, 4 * q + 2), PX(s, 4 * q + 3));
  }
  if (tid < TS_B * TS_B) {
    const int a = tid / TS_B, c = tid % TS_B;
    Tw[(int64_t)b * TS_B * TS_B + tid] = Ts[a][c];
  }
#undef PX
}

// band extraction: AB[b][c][d] = A[c+d][c] for d <= 16 (c + d < n), 0 for
// 16 < d < 32 and for the padding columns c >= n
__global__ void sb_extract_kernel(const float* __restrict__ A, int64_t sA, int ld, int n,
                                  float* __restrict__ AB, int64_t sAB, int ncols) {
  const int b = blockIdx.y;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ncols * 2 * TS_B) return;
  const int c = e / (2 * TS_B), d = e % (2 * TS_B);
  float v = 0.f;
  if (c < n && d <= TS_B && c + d < n) v = A[(int64_t)b * sA + (int64_t)(c + d) * ld + c];
  AB[(int64_t)b * sAB + e] = v;
}

typedef float v4f __attribute__((ext_vector_type(4)));

// ---- two-sided trailing update of panel p, A22 = A[p+16:, p+16:] (m x m,
// leading dimension ld), Q_p = I - V T V^T:
//   Y = A22 U (U = V T), S = V^T Y, Ms = sym(T^T S), W = Y - 1/2 V Ms,
//   A22 -= V W^T + W V^T.

// Y (split-K partials) and the partial S = V^T Y of 64 rows, one 16-row
// strip per wave on v_mfma_f32_16x16x4_f32.  grid (ceil(m/64), KS, batch).
__global__ void __launch_bounds__(256) sb_symm_kernel(
    const float* __restrict__ A, int64_t sA, int ld, int n, int p, const float* __restrict__ Uw,
    const float* __restrict__ Vw, int64_t sVU, int kchunk, float* __restrict__ Ypart,
    float* __restrict__ Spart, int nparts) {
  const int b = blockIdx.z, split = blockIdx.y, blk = blockIdx.x;
  const int KS = gridDim.y;
  const int m = n - p - TS_B;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int li = l & 15, lk = l >> 4;
  const float* A22 = A + (int64_t)b * sA + (int64_t)(p + TS_B) * ld + (p + TS_B);
  const float* U = Uw + (int64_t)b * sVU;
  const float* V = Vw + (int64_t)b * sVU;
  const int r0 = blk * 64 + 16 * w;
  const int row = r0 + li;
  const int k_lo = split * kchunk, k_hi = min(m, k_lo + kchunk);
  v4f acc = {0.f, 0.f, 0.f, 0.f};
  const float* arow = A22 + (int64_t)row * ld;
  const bool rok = row < m;
  for (int kk = k_lo; kk < k_hi; kk += 16) {
    const int k4 = kk + 4 * lk;
    float a[4], u[4];
    if (rok && k4 + 3 < k_hi) {
      const float4 x = *reinterpret_cast<const float4*>(arow + k4);
      a[0] = x.x; a[1] = x.y; a[2] = x.z; a[3] = x.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] = (rok && k4 + e < k_hi) ? arow[k4 + e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) u[e] = k4 + e < k_hi ? U[(int64_t)(k4 + e) * TS_B + li] : 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], u[e], acc, 0, 0, 0);
  }
  // acc[i] = Y[r0 + 4 lk + i][li]
  float* Yp = Ypart + ((int64_t)split * gridDim.z + b) * (int64_t)n * TS_B;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + 4 * lk + i;
    if (r < m) Yp[(int64_t)r * TS_B + li] = acc[i];
  }
  // partial S = V_rows^T Y_rows: A operand V^T[t = li][row 4 lk + e], B = acc[e]
  v4f sacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int r = r0 + 4 * lk + e;
    const float v = r < m ? V[(int64_t)r * TS_B + li] : 0.f;
    sacc = __builtin_amdgcn_mfma_f32_16x16x4f32(v, acc[e], sacc, 0, 0, 0);
  }
  __shared__ float sred[4][TS_B * TS_B];
#pragma unroll
  for (int i = 0; i < 4; ++i) sred[w][(4 * lk + i) * TS_B + li] = sacc[i];
  __syncthreads();
  const int part = blk * KS + split;
  if (threadIdx.x < TS_B * TS_B) {
    const int e = threadIdx.x;
    Spart[((int64_t)b * nparts + part) * TS_B * TS_B + e] =
        (sred[0][e] + sred[1][e]) + (sred[2][e] + sred[3][e]);
  }
}

// Ms = sym(T^T S), S = sum of the partials in a fixed order.  grid (batch), 1024
__global__ void __launch_bounds__(1024) sb_sred_kernel(const float* __restrict__ Spart,
                                                       int nparts, const float* __restrict__ Tw,
                                                       float* __restrict__ Ms) {
  const int b = blockIdx.x;
  const int e = threadIdx.x & 255, q = threadIdx.x >> 8;
  __shared__ float part[4][TS_B * TS_B];
  __shared__ float S[TS_B][TS_B + 1];
  __shared__ float M[TS_B][TS_B + 1];
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  const float* sp = Spart + (int64_t)b * nparts * TS_B * TS_B;
  int i = q;
  for (; i + 12 < nparts; i += 16) {  // four independent loads in flight
    s0 += sp[(int64_t)i * TS_B * TS_B + e];
    s1 += sp[(int64_t)(i + 4) * TS_B * TS_B + e];
    s2 += sp[(int64_t)(i + 8) * TS_B * TS_B + e];
    s3 += sp[(int64_t)(i + 12) * TS_B * TS_B + e];
  }
  for (; i < nparts; i += 4) s0 += sp[(int64_t)i * TS_B * TS_B + e];
  part[q][e] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (threadIdx.x < 256) S[e / TS_B][e % TS_B] = (part[0][e] + part[1][e]) + (part[2][e] + part[3][e]);
  __syncthreads();
  const float* T = Tw + (int64_t)b * TS_B * TS_B;
  if (threadIdx.x < 256) {
    const int t = e / TS_B, c = e % TS_B;
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < TS_B; ++k) a += T[k * TS_B + t] * S[k][c];
    M[t][c] = a;
  }
  __syncthreads();
  if (threadIdx.x < 256) {
    const int t = e / TS_B, c = e % TS_B;
    Ms[(int64_t)b * TS_B * TS_B + e] = 0.5f * (M[t][c] + M[c][t]);
  }
}

// W = Y - 1/2 V Ms (Y = sum of the split partials), once per row.
// grid (ceil(m/256), batch), 256 threads
__global__ void __launch_bounds__(256) sb_w_kernel(int n, int p, const float* __restrict__ Vw,
                                                   int64_t sVU, const float* __restrict__ Ypart,
                                                   int KS, const float* __restrict__ Ms,
                                                   float* __restrict__ Ww) {
  const int b = blockIdx.y;
  const int m = n - p - TS_B;
  __shared__ float Msh[TS_B][TS_B + 1];
  Msh[threadIdx.x / TS_B][threadIdx.x % TS_B] = Ms[(int64_t)b * TS_B * TS_B + threadIdx.x];
  __syncthreads();
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= m) return;
  float v[TS_B], y[TS_B];
  const float4* vr = reinterpret_cast<const float4*>(Vw + (int64_t)b * sVU + (int64_t)r * TS_B);
#pragma unroll
  for (int q = 0; q < TS_B / 4; ++q) {
    const float4 x = vr[q];
    v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
    y[4 * q] = y[4 * q + 1] = y[4 * q + 2] = y[4 * q + 3] = 0.f;
  }
  for (int sp = 0; sp < KS; ++sp) {
    const float4* yr = reinterpret_cast<const float4*>(
        Ypart + ((int64_t)sp * gridDim.y + b) * (int64_t)n * TS_B + (int64_t)r * TS_B);
#pragma unroll
    for (int q = 0; q < TS_B / 4; ++q) {
      const float4 x = yr[q];
      y[4 * q] += x.x; y[4 * q + 1] += x.y; y[4 * q + 2] += x.z; y[4 * q + 3] += x.w;
    }
  }
  float4* wr = reinterpret_cast<float4*>(Ww + (int64_t)b * sVU + (int64_t)r * TS_B);
#pragma unroll
  for (int q = 0; q < TS_B / 4; ++q) {
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int t = 4 * q + e;
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < TS_B; ++k) a += v[k] * Msh[k][t];
      o[e] = y[t] - 0.5f * a;
    }
    wr[q] = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// A22 -= V W^T + W V^T on 64 x 64 tiles.
// grid (ceil(m/64) col tiles, ceil(m/64) row tiles, batch), 256 threads
__global__ void __launch_bounds__(256) sb_upd_kernel(
    float* __restrict__ A, int64_t sA, int ld, int n, int p, const float* __restrict__ Vw,
    int64_t sVU, const float* __restrict__ Ww, int ctile0) {
  const int b = blockIdx.z;
  const int m = n - p - TS_B;
  const int R0 = blockIdx.y * 64, C0 = (blockIdx.x + ctile0) * 64;
  const int tid = threadIdx.x;
  __shared__ __attribute__((aligned(16))) float Vr[64][TS_B + 4], Wr[64][TS_B + 4];
  __shared__ __attribute__((aligned(16))) float Vc[64][TS_B + 4], Wc[64][TS_B + 4];
  const float* V = Vw + (int64_t)b * sVU;
  const float* W = Ww + (int64_t)b * sVU;
  // this thread's 4 x 4 block of the tile (rows R0 + 4 ty + i, columns
  // C0 + 4 tx .. +3: 16-B loads), in flight while V / W are staged
  const int ty = tid >> 4, tx = tid & 15;
  float* A22 = A + (int64_t)b * sA + (int64_t)(p + TS_B) * ld + (p + TS_B);
  const int cb = C0 + 4 * tx;
  const bool cfull = cb + 3 < m;
  float4 a4[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = R0 + 4 * ty + i;
    a4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < m) {
      const float* ar = A22 + (int64_t)r * ld + cb;
      if (cfull) {
        a4[i] = *reinterpret_cast<const float4*>(ar);
      } else {
        if (cb < m) a4[i].x = ar[0];
        if (cb + 1 < m) a4[i].y = ar[1];
        if (cb + 2 < m) a4[i].z = ar[2];
      }
    }
  }
  for (int e = tid; e < 2 * 64 * (TS_B / 4); e += 256) {
    const int side = e / (64 * (TS_B / 4)), rr = (e / (TS_B / 4)) % 64, q = e % (TS_B / 4);
    const int r = (side ? C0 : R0) + rr;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f), w = v;
    if (r < m) {
      v = reinterpret_cast<const float4*>(V + (int64_t)r * TS_B)[q];
      w = reinterpret_cast<const float4*>(W + (int64_t)r * TS_B)[q];
    }
    if (side) {
      *reinterpret_cast<float4*>(&Vc[rr][4 * q]) = v;
      *reinterpret_cast<float4*>(&Wc[rr][4 * q]) = w;
    } else {
      *reinterpret_cast<float4*>(&Vr[rr][4 * q]) = v;
      *reinterpret_cast<float4*>(&Wr[rr][4 * q]) = w;
    }
  }
  __syncthreads();
  float acc[4][4] = {};
#pragma unroll
  for (int t4 = 0; t4 < TS_B; t4 += 4) {
    float4 vr[4], wr[4], vc[4], wc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      vr[i] = *reinterpret_cast<const float4*>(&Vr[4 * ty + i][t4]);
      wr[i] = *reinterpret_cast<const float4*>(&Wr[4 * ty + i][t4]);
      vc[i] = *reinterpret_cast<const float4*>(&Vc[4 * tx + i][t4]);
      wc[i] = *reinterpret_cast<const float4*>(&Wc[4 * tx + i][t4]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] += (vr[i].x * wc[j].x + wr[i].x * vc[j].x) + (vr[i].y * wc[j].y + wr[i].y * vc[j].y) +
                     (vr[i].z * wc[j].z + wr[i].z * vc[j].z) + (vr[i].w * wc[j].w + wr[i].w * vc[j].w);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = R0 + 4 * ty + i;
    if (r >= m) continue;
    float* ar = A22 + (int64_t)r * ld + cb;
    const float4 o = make_float4(a4[i].x - acc[i][0], a4[i].y - acc[i][1], a4[i].z - acc[i][2],
                                 a4[i].w - acc[i][3]);
    if (cfull) {
      *reinterpret_cast<float4*>(ar) = o;
    } else {
      if (cb < m) ar[0] = o.x;
      if (cb + 1 < m) ar[1] = o.y;
      if (cb + 2 < m) ar[2] = o.z;
    }
  }
}

}  // namespace

void sb_panel_qr(float* A, int64_t sA, int ld, int n, int p, int batch, float* Vw,
                 float* Uw, int64_t sVU, float* tau1, int64_t sTau, float* Tw,
                 hipStream_t stream) {
  const int m = n - p - TS_B;
  if (m <= 0 || batch <= 0) return;
  const int rpt = (int)ceil_div(m, QR_T);
#define KFAC_SBQR(R)                                                                   \
  hipLaunchKernelGGL(sb_qr_kernel<R>, dim3(batch), dim3(QR_T), 0, stream, A, sA, ld, n, p, \
                     Vw, Uw, sVU, tau1, sTau, Tw)
  switch (rpt) {
    case 1: KFAC_SBQR(1); break;
    case 2: KFAC_SBQR(2); break;
    case 3: KFAC_SBQR(3); break;
    case 4: KFAC_SBQR(4); break;
    case 5: KFAC_SBQR(5); break;
    default: break;  // host checks n <= twostage_max_n()
  }
#undef KFAC_SBQR
}

void sb_extract(const float* A, int64_t sA, int ld, int n, int batch, float* AB, int64_t sAB,
                int ncols, hipStream_t stream) {
  const int total = ncols * 2 * TS_B;
  hipLaunchKernelGGL(sb_extract_kernel, dim3((unsigned)ceil_div(total, 256), batch), dim3(256),
                     0, stream, A, sA, ld, n, AB, sAB, ncols);
}

// Y / S partials, Ms, tile update for panel p.  Ypart [KS][batch][n][16],
// Spart [batch][nparts][16][16], Ms [batch][16][16]; returns nothing, queues 3
// launches on `stream`.
int sb_update_splits(int m, int batch) {
  const int nblk = (int)ceil_div(m, 64);
  int ks = (int)ceil_div(512, (int64_t)nblk * batch);
  ks = ks < 1 ? 1 : (ks > 8 ? 8 : ks);
  return ks;
}

// front part of panel p's update on `stream`: Y / S partials, Ms, W and the
// first 64 columns of the trailing matrix (they hold the next panel, so the
// next panel QR can start); sb_update_back updates the other columns (on a
// second stream, overlapping that QR)
void sb_update_front(float* A, int64_t sA, int ld, int n, int p, int batch, const float* Vw,
                     const float* Uw, int64_t sVU, const float* Tw, float* Ypart, float* Spart,
                     float* Ms, float* Ww, hipStream_t stream) {
  const int m = n - p - TS_B;
  if (m <= 0 || batch <= 0) return;
  const int nblk = (int)ceil_div(m, 64);
  const int ks = sb_update_splits(m, batch);
  const int kchunk = (int)ceil_div(ceil_div(m, ks), 16) * 16;
  const int nparts = nblk * ks;
  hipLaunchKernelGGL(sb_symm_kernel, dim3(nblk, ks, batch), dim3(256), 0, stream, A, sA, ld, n,
                     p, Uw, Vw, sVU, kchunk, Ypart, Spart, nparts);
  hipLaunchKernelGGL(sb_sred_kernel, dim3(batch), dim3(1024), 0, stream, Spart, nparts, Tw, Ms);
  hipLaunchKernelGGL(sb_w_kernel, dim3((unsigned)ceil_div(m, 256), batch), dim3(256), 0, stream,
                     n, p, Vw, sVU, Ypart, ks, Ms, Ww);
  hipLaunchKernelGGL(sb_upd_kernel, dim3(1, nblk, batch), dim3(256), 0, stream, A, sA, ld, n, p,
                     Vw, sVU, Ww, 0);
}

// true when there are columns left for sb_update_back
bool sb_update_back(float* A, int64_t sA, int ld, int n, int p, int batch, const float* Vw,
                    int64_t sVU, const float* Ww, hipStream_t stream) {
  const int m = n - p - TS_B;
  if (m <= 0 || batch <= 0) return false;
  const int nblk = (int)ceil_div(m, 64);
  if (nblk < 2) return false;
  hipLaunchKernelGGL(sb_upd_kernel, dim3(nblk - 1, nblk, batch), dim3(256), 0, stream, A, sA, ld,
                     n, p, Vw, sVU, Ww, 1);
  return true;
}

}  // namespace kfac
