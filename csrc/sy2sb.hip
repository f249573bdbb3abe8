// K-HIP-3, two-stage eigensolver, stage 1: dense symmetric -> band (width 16).
//
// A = Q1 B Q1^T with B banded (|i - j| <= 16).  Panel p (columns p..p+15,
// rows p+16..n-1, m = n - p - 16 rows) is factored P = Q_p R by Householder
// QR; the trailing matrix is then updated two-sidedly,
//   A22 <- Q_p^T A22 Q_p,  Q_p = I - V T V^T,
// with level-3 operations only (Y = A22 V T, W = Y - 1/2 V sym(T^T V^T Y),
// A22 -= V W^T + W V^T: batched library GEMMs driven from
// csrc/twostage_host.cpp).  The one-stage Householder tridiagonalisation
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
//   A lower panel  <- R (upper triangular 16 x 16) and zeros below: the band;
//   A row p+a      <- column a of the factored panel (R^T in the band, the
//                     reflector v_a beyond it: v_a[p+16+a] = 1 implicit), the
//                     layout the blocked back-transform reads (offset 16);
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

// block-wide sums of 16 per-thread values; every thread receives the totals
__device__ __forceinline__ void block_sum16(float (&v)[TS_B], float* red, float* tot) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < TS_B; ++c) {
    const float s = wave_sum_uniform(v[c]);
    if (l == 0) red[w * TS_B + c] = s;
  }
  __syncthreads();
  if (threadIdx.x < TS_B) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < QR_W; ++q) s += red[q * TS_B + threadIdx.x];
    tot[threadIdx.x] = s;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < TS_B; ++c) v[c] = tot[c];
}

__device__ __forceinline__ float block_sum1(float v, float* red, float* tot) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const float s = wave_sum_uniform(v);
  if (l == 0) red[w] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < QR_W; ++q) t += red[q];
    tot[0] = t;
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
  __shared__ float red[QR_W * TS_B];
  __shared__ float tot[TS_B];
  __shared__ float Ts[TS_B][TS_B + 1];
  __shared__ float alpha_s;

  float P[RPT][TS_B];
#pragma unroll
  for (int s = 0; s < RPT; ++s) {
    const int i = tid + QR_T * s;
    if (i < m) {
      const float4* row = reinterpret_cast<const float4*>(Ab + (int64_t)(p + TS_B + i) * ld + p);
#pragma unroll
      for (int q = 0; q < TS_B / 4; ++q) {
        const float4 x = row[q];
        P[s][4 * q] = x.x;
        P[s][4 * q + 1] = x.y;
        P[s][4 * q + 2] = x.z;
        P[s][4 * q + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int c = 0; c < TS_B; ++c) P[s][c] = 0.f;
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
        if (i > t && i < m) part += P[s][t] * P[s][t];
      }
      if (tid == t) alpha_s = P[0][t];
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
        vv[s] = i == t ? 1.f : ((i > t && i < m) ? P[s][t] * scale : 0.f);
      }
      // ---- u_c = v^T P[:, c]: trailing columns (c > t) for the update,
      // earlier columns (c < t: the stored reflectors) for T
      float u[TS_B];
#pragma unroll
      for (int c = 0; c < TS_B; ++c) {
        float a = 0.f;
        if (c != t) {
#pragma unroll
          for (int s = 0; s < RPT; ++s) a += vv[s] * P[s][c];
        }
        u[c] = a;
      }
      block_sum16(u, red, tot);
#pragma unroll
      for (int c = t + 1; c < TS_B; ++c) {
        const float f = tau * u[c];
#pragma unroll
        for (int s = 0; s < RPT; ++s) P[s][c] -= f * vv[s];
      }
#pragma unroll
      for (int s = 0; s < RPT; ++s) {
        const int i = tid + QR_T * s;
        if (i == t) P[s][t] = beta;
        else if (i > t) P[s][t] = vv[s];
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
    for (int a = 0; a < TS_B; ++a) v[a] = i > a ? P[s][a] : (i == a ? 1.f : 0.f);
    if (i >= bb) {
      // rows past the last reflector's start only exist when m > 16
    }
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
    // lower panel: R on and above the diagonal, zeros below (the band)
    float4* arow = reinterpret_cast<float4*>(Ab + (int64_t)(p + TS_B + i) * ld + p);
#pragma unroll
    for (int q = 0; q < TS_B / 4; ++q) {
      float r4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) r4[e] = i <= 4 * q + e ? P[s][4 * q + e] : 0.f;
      arow[q] = make_float4(r4[0], r4[1], r4[2], r4[3]);
    }
    // row storage: A[p+a][p+16+i] = factored column a (R^T, then v_a)
#pragma unroll
    for (int a = 0; a < TS_B; ++a) Ab[(int64_t)(p + a) * ld + p + TS_B + i] = P[s][a];
  }
  if (tid < TS_B * TS_B) {
    const int a = tid / TS_B, c = tid % TS_B;
    Tw[(int64_t)b * TS_B * TS_B + tid] = Ts[a][c];
  }
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

}  // namespace kfac
