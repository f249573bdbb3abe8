// K-HIP-3, last stage: batched symmetric TRIDIAGONAL eigensolver by Cuppen's
// divide and conquer with Gu-Eisenstat eigenvectors.  Replaces rocSOLVER's
// stedc behind the native Householder reduction (csrc/sytrd.hip), so an eigen
// refresh runs no library eigensolver (reference: torch.linalg.eigh,
// kfac/layers/eigen.py:294-347).  The float64 CPU reference of every step is
// distributed_kfac_pytorch_amd/ops/tridiag.py; the driver (padding to a
// uniform tree, leaves on the LDS Jacobi kernel, one batched GEMM per level)
// is csrc/tridiag_host.cpp.
//
// One merge level = every subproblem of size m = 2h of every matrix:
//   dc_sort     merge the children's ascending eigenvalues (one binary search
//               per element), gather z = [Q1 last row, sgn Q2 first row]/sqrt2,
//               deflation tolerance;
//   dc_deflate  LAPACK slaed2's two deflation tests in one sequential walk
//               (small rho~|z_i|; Givens-combined close pairs), chunk-staged
//               through LDS;
//   dc_secular  one thread per root of 1 + rho~ sum z^2/(d - lam) in float64,
//               each root kept as (pole, tau) so d_i - lam_j never cancels;
//               safeguarded two-pole rational iteration;
//   dc_zhat     Gu-Eisenstat z^ from the roots (pairwise-ratio products);
//   dc_vectors  u_j = z^ / (d - lam_j) normalised, written as the columns of W
//               (row = child coordinate, column = output position after the
//               final ascending sort), deflated entries as unit columns;
//   dc_rotate   the deflation rotations folded into W's rows (reverse order);
// then Q_parent = diag(Q1, Q2) W is one batched GEMM (host).
#include "common.h"

namespace kfac {

namespace {

constexpr int DC_T = 256;
constexpr int DC_CH = 1024;  // entries per LDS chunk of the streamed passes
constexpr double EPS64 = 2.220446049250313e-16;

__device__ __forceinline__ double block_max_d(double v, double* red) {
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  double r = red[0];
  for (int t = 1; t < DC_T / 64; ++t) r = fmax(r, red[t]);
  return r;
}

// number of a[0, len) strictly below x / at most x (a ascending)
__device__ __forceinline__ int count_lt(const double* a, int len, double x) {
  int lo = 0, hi = len;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int count_le(const double* a, int len, double x) {
  int lo = 0, hi = len;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Leaves: dense [leaf x leaf] blocks of the padded tridiagonal with the split
// corrections d -= |e| on both sides of every leaf boundary.  grid: blocks.
__global__ void __launch_bounds__(64) dc_leaves_kernel(
    const float* __restrict__ d, const float* __restrict__ e, int n_pad, int leaf,
    float* __restrict__ out) {
  const int blk = blockIdx.x;
  const int nl = n_pad / leaf;
  const int b = blk / nl, l0 = (blk % nl) * leaf;
  const float* db = d + (int64_t)b * n_pad;
  const float* eb = e + (int64_t)b * (n_pad - 1);
  float* o = out + (int64_t)blk * leaf * leaf;
  for (int t = threadIdx.x; t < leaf * leaf; t += 64) o[t] = 0.f;
  __syncthreads();
  for (int i = threadIdx.x; i < leaf; i += 64) {
    const int r = l0 + i;
    float dv = db[r];
    if (i == 0 && r > 0) dv -= fabsf(eb[r - 1]);
    if (i == leaf - 1 && r < n_pad - 1) dv -= fabsf(eb[r]);
    o[i * leaf + i] = dv;
    if (i < leaf - 1) {
      o[i * leaf + i + 1] = eb[r];
      o[(i + 1) * leaf + i] = eb[r];
    }
  }
}

// grid: G subproblems (g = matrix * S + s).  Dprev [G, m] (child 1 | child 2,
// each ascending), Qprev [2G, h, h].  Writes sd / sz / perm in sorted order
// and scal[g] = {rho~, tol, 0, 0}.
__global__ void __launch_bounds__(DC_T) dc_sort_kernel(
    const double* __restrict__ Dprev, const float* __restrict__ Qprev,
    const float* __restrict__ e_pad, int n_pad, int h, int S,
    double* __restrict__ sd, double* __restrict__ sz, int* __restrict__ perm,
    double* __restrict__ scal) {
  extern __shared__ double sh[];  // m doubles: the children's eigenvalues
  __shared__ double red[DC_T / 64];
  const int g = blockIdx.x, m = 2 * h;
  const int b = g / S, s = g % S;
  const double* D = Dprev + (int64_t)g * m;
  for (int i = threadIdx.x; i < m; i += DC_T) {
    const double v = D[i];
    sh[i] = v == v ? v : __builtin_huge_val();
  }
  const float beta = e_pad[(int64_t)b * (n_pad - 1) + (int64_t)s * m + h - 1];
  const double sgn = beta >= 0.f ? 1.0 : -1.0;
  const double rho = 2.0 * fabs((double)beta);
  __syncthreads();
  const float* Q1 = Qprev + (int64_t)(2 * g) * h * h;
  const float* Q2 = Q1 + (int64_t)h * h;
  const double r2 = 0.70710678118654752440;
  double mx_d = 0.0, mx_z = 0.0;
  const int64_t base = (int64_t)g * m;
  for (int i = threadIdx.x; i < h; i += DC_T) {
    const double a = sh[i];
    const int p = i + count_lt(sh + h, h, a);
    const double z = (double)Q1[(int64_t)(h - 1) * h + i] * r2;
    sd[base + p] = a;
    sz[base + p] = z;
    perm[base + p] = i;
    mx_d = fmax(mx_d, fabs(a));
    mx_z = fmax(mx_z, fabs(z));
  }
  for (int i = threadIdx.x; i < h; i += DC_T) {
    const double a = sh[h + i];
    const int p = i + count_le(sh, h, a);
    const double z = sgn * (double)Q2[i] * r2;
    sd[base + p] = a;
    sz[base + p] = z;
    perm[base + p] = h + i;
    mx_d = fmax(mx_d, fabs(a));
    mx_z = fmax(mx_z, fabs(z));
  }
  mx_d = block_max_d(mx_d, red);
  mx_z = block_max_d(mx_z, red);
  if (threadIdx.x == 0) {
    // LAPACK slaed2: tol = 8 eps max(|d|, |rho z|) -- eps of the fp32 data
    const double eps32 = 5.9604644775390625e-08;
    scal[(int64_t)g * 4 + 0] = rho;
    scal[(int64_t)g * 4 + 1] = 8.0 * eps32 * fmax(mx_d, rho * mx_z);
  }
}

// grid: G.  Sequential deflation walk (thread 0) over LDS-staged chunks.
// isnd[r] = rank among the survivors or -1; ndidx[rank] = r; rot = (p, i)
// pairs with (c, s); cnt[g] = {K, nrot}; vals[r] = final value of deflated r.
__global__ void __launch_bounds__(DC_T) dc_deflate_kernel(
    int m, double* __restrict__ sd, double* __restrict__ sz,
    const double* __restrict__ scal, int* __restrict__ isnd, int* __restrict__ ndidx,
    int* __restrict__ rot_idx, double* __restrict__ rot_cs, int* __restrict__ cnt,
    double* __restrict__ vals) {
  __shared__ double cd[DC_CH], cz[DC_CH];
  const int g = blockIdx.x;
  const int64_t base = (int64_t)g * m;
  const double rho = scal[(int64_t)g * 4 + 0], tol = scal[(int64_t)g * 4 + 1];
  int K = 0, p = -1, nrot = 0;
  double dp = 0.0, zp = 0.0;
  for (int c0 = 0; c0 < m; c0 += DC_CH) {
    const int len = min(DC_CH, m - c0);
    __syncthreads();
    for (int t = threadIdx.x; t < len; t += DC_T) {
      cd[t] = sd[base + c0 + t];
      cz[t] = sz[base + c0 + t];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int t = 0; t < len; ++t) {
        const int i = c0 + t;
        const double di = cd[t], zi = cz[t];
        if (rho * fabs(zi) <= tol) {
          isnd[base + i] = -1;
          continue;
        }
        if (p >= 0) {
          double s = zp, c = zi;
          const double tt = hypot(c, s);
          c /= tt;
          s = -s / tt;
          if (fabs((di - dp) * c * s) <= tol) {
            // Givens: z_p -> 0 (deflated), z_i -> tt
            sd[base + p] = dp * c * c + di * s * s;
            sz[base + p] = 0.0;
            isnd[base + p] = -1;
            rot_idx[(base + nrot) * 2 + 0] = p;
            rot_idx[(base + nrot) * 2 + 1] = i;
            rot_cs[(base + nrot) * 2 + 0] = c;
            rot_cs[(base + nrot) * 2 + 1] = s;
            ++nrot;
            isnd[base + i] = K - 1;
            ndidx[base + K - 1] = i;
            dp = dp * s * s + di * c * c;
            zp = tt;
            p = i;
            continue;
          }
          sd[base + p] = dp;
          sz[base + p] = zp;
        }
        isnd[base + i] = K;
        ndidx[base + K] = i;
        ++K;
        p = i;
        dp = di;
        zp = zi;
      }
    }
  }
  if (threadIdx.x == 0) {
    if (p >= 0) {
      sd[base + p] = dp;
      sz[base + p] = zp;
    }
    cnt[g * 2 + 0] = K;
    cnt[g * 2 + 1] = nrot;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < m; r += DC_T)
    if (isnd[base + r] < 0) vals[base + r] = sd[base + r];
}

// psi / phi sums over the survivors at lam = dn[o] + t, chunk-streamed
// through LDS; every thread of the block must call it (lockstep passes).
struct SecSums {
  double psi, dpsi, phi, dphi, zsum;
};

__device__ __forceinline__ SecSums sec_sums(const double* __restrict__ sd,
                                            const double* __restrict__ sz,
                                            const int* __restrict__ ndidx, int64_t base,
                                            int K, int j, double dorg, double t, bool act,
                                            double* cd, double* cz2) {
  SecSums r{0.0, 0.0, 0.0, 0.0, 0.0};
  for (int c0 = 0; c0 < K; c0 += DC_CH) {
    const int len = min(DC_CH, K - c0);
    __syncthreads();
    for (int q = threadIdx.x; q < len; q += DC_T) {
      const int idx = ndidx[base + c0 + q];
      cd[q] = sd[base + idx];
      const double z = sz[base + idx];
      cz2[q] = z * z;
    }
    __syncthreads();
    for (int q = 0; q < len; ++q) r.zsum += cz2[q];
    if (act) {
      for (int q = 0; q < len; ++q) {
        const int i = c0 + q;
        const double del = (cd[q] - dorg) - t;
        const double rr = 1.0 / del;
        const double w = cz2[q] * rr;
        if (i <= j) {
          r.psi += w;
          r.dpsi += w * rr;
        } else {
          r.phi += w;
          r.dphi += w * rr;
        }
      }
    }
  }
  return r;
}

// zero of c + s1/(a1 - y) + s2/(a2 - y) (y = step from t; poles a1 < 0 < a2
// relative to t), Gragg's two-pole model of f; Newton if degenerate
__device__ __forceinline__ double two_pole(double t, double f, double rho, const SecSums& S,
                                          double p1, double p2, bool last) {
  const double a1 = p1 - t;
  const double s1 = rho * S.dpsi * a1 * a1;
  if (last) {
    const double c = f - s1 / a1;
    return c != 0.0 ? p1 + s1 / c : t;
  }
  const double a2 = p2 - t;
  const double s2 = rho * S.dphi * a2 * a2;
  const double c = f - s1 / a1 - s2 / a2;
  const double qa = c, qb = -(c * (a1 + a2) + s1 + s2), qc = c * a1 * a2 + s1 * a2 + s2 * a1;
  const double lo = fmin(a1, a2), hi = fmax(a1, a2);
  if (qa != 0.0) {
    double disc = qb * qb - 4.0 * qa * qc;
    if (disc < 0.0) disc = 0.0;
    const double sq = sqrt(disc);
    const double qq = -0.5 * (qb + copysign(sq, qb));
    if (qq != 0.0) {
      const double y = qc / qq;
      if (y > lo && y < hi) return t + y;
    }
    const double y = qq / qa;
    if (y > lo && y < hi) return t + y;
  } else if (qb != 0.0) {
    const double y = -qc / qb;
    if (y > lo && y < hi) return t + y;
  }
  const double der = rho * (S.dpsi + S.dphi);
  return der > 0.0 ? t - f / der : t;
}

// grid: (G, ceil(m / DC_T)).  tau[j] > 0: lam_j = dn[j] + tau (origin j);
// tau[j] < 0: lam_j = dn[j+1] + tau.
__global__ void __launch_bounds__(DC_T) dc_secular_kernel(
    int m, const double* __restrict__ sd, const double* __restrict__ sz,
    const int* __restrict__ ndidx, const int* __restrict__ cnt,
    const double* __restrict__ scal, double* __restrict__ tau, double* __restrict__ vals) {
  __shared__ double cd[DC_CH], cz2[DC_CH];
  const int g = blockIdx.x;
  const int K = cnt[g * 2 + 0];
  const int j = blockIdx.y * DC_T + threadIdx.x;
  if ((int)(blockIdx.y * DC_T) >= K) return;  // uniform per block
  const int64_t base = (int64_t)g * m;
  const double rho = scal[(int64_t)g * 4 + 0];
  const bool act0 = j < K;
  const bool last = j == K - 1;
  double dj = 0.0, dj1 = 0.0;
  if (act0) {
    dj = sd[base + ndidx[base + j]];
    dj1 = last ? dj : sd[base + ndidx[base + j + 1]];
  }
  // probe pass (every thread): |z|^2 of the survivors, and f at the midpoint
  // of each interval (d_j, d_j+1) to pick the closer pole as origin
  const double mid = (act0 && !last) ? 0.5 * (dj1 - dj) : 0.0;
  SecSums S = sec_sums(sd, sz, ndidx, base, K, j, dj, mid, act0 && !last, cd, cz2);
  const double zsum = S.zsum;
  bool act = act0;
  int o = j;
  double dorg = dj, t, lo, hi;
  if (!last) {
    const double f = 1.0 + rho * (S.psi + S.phi);
    if (f > 0.0) {
      o = j; dorg = dj; lo = 0.0; hi = mid; t = mid;
    } else {
      o = j + 1; dorg = dj1; lo = -mid; hi = 0.0; t = -mid;
    }
    if (act) {
      double tn = two_pole(t, f, rho, S, dj - dorg, dj1 - dorg, false);
      if (!(tn > lo && tn < hi)) tn = 0.5 * (lo + hi);
      t = tn;
    }
  } else {
    lo = 0.0;
    hi = rho * zsum;
    t = 0.5 * hi;
  }
  for (int it = 0; it < 80; ++it) {
    const int more = __syncthreads_or(act ? 1 : 0);
    if (!more) break;
    S = sec_sums(sd, sz, ndidx, base, K, j, dorg, t, act, cd, cz2);
    if (!act) continue;
    const double f = 1.0 + rho * (S.psi + S.phi);
    if (f == 0.0) { act = false; continue; }
    if (f > 0.0) hi = t; else lo = t;
    const double scale = fabs(dorg) + fabs(t);
    if (hi - lo <= 4.0 * EPS64 * scale ||
        fabs(f) <= 8.0 * K * EPS64 * (1.0 + rho * (fabs(S.psi) + fabs(S.phi)))) {
      act = false;
      continue;
    }
    const double p1 = dj - dorg, p2 = dj1 - dorg;
    double tn = two_pole(t, f, rho, S, p1, p2, last);
    if (!(tn > lo && tn < hi)) tn = 0.5 * (lo + hi);
    if (tn == t) { act = false; continue; }
    t = tn;
  }
  if (act0) {
    // a converged root never sits on its pole; keep the sign convention
    if (o == j && t <= 0.0) t = 0.5 * hi;
    if (o != j && t >= 0.0) t = 0.5 * lo;
    tau[base + j] = t;
    vals[base + ndidx[base + j]] = dorg + t;
  }
}

// grid: (G, ceil(m / DC_T)).  z^_i = sign(z_i) sqrt(prod_j (lam_j - d_i) /
// (rho prod_{j != i} (d_j - d_i))), paired as ratios.
__global__ void __launch_bounds__(DC_T) dc_zhat_kernel(
    int m, const double* __restrict__ sd, const double* __restrict__ sz,
    const int* __restrict__ ndidx, const int* __restrict__ cnt,
    const double* __restrict__ scal, const double* __restrict__ tau,
    double* __restrict__ zh) {
  __shared__ double cd[DC_CH + 1], ct[DC_CH];
  const int g = blockIdx.x;
  const int K = cnt[g * 2 + 0];
  if ((int)(blockIdx.y * DC_T) >= K) return;
  const int i = blockIdx.y * DC_T + threadIdx.x;
  const bool act = i < K;
  const int64_t base = (int64_t)g * m;
  const double rho = scal[(int64_t)g * 4 + 0];
  double di = 0.0, prod = 1.0;
  if (act) {
    di = sd[base + ndidx[base + i]];
    const double ti = tau[base + i];
    // origin j+1 only when tau < 0 AND a next pole exists (NaN-safe: a
    // non-finite factor must give non-finite results, never a stray index)
    const double doi = (ti > 0.0 || i == K - 1) ? di : sd[base + ndidx[base + i + 1]];
    prod = ((doi - di) + ti) / rho;
  }
  for (int c0 = 0; c0 < K; c0 += DC_CH) {
    const int len = min(DC_CH, K - c0);
    __syncthreads();
    for (int q = threadIdx.x; q <= len; q += DC_T) {
      const int jj = c0 + q;
      if (jj < K) cd[q] = sd[base + ndidx[base + jj]];
      if (q < len) ct[q] = tau[base + jj];
    }
    __syncthreads();
    if (act) {
      for (int q = 0; q < len; ++q) {
        const int jj = c0 + q;
        if (jj == i) continue;
        const double tj = ct[q];
        const double dorg = (tj > 0.0 || jj == K - 1) ? cd[q] : cd[q + 1];
        prod *= ((dorg - di) + tj) / (cd[q] - di);
      }
    }
  }
  if (act) {
    const double z = sz[base + ndidx[base + i]];
    zh[base + i] = copysign(sqrt(fmax(prod, 0.0)), z);
  }
}

// grid: (G, ceil(m / DC_T)).  Columns of W (zeroed by the host): root j ->
// column outpos[ndidx[j]], rows perm[ndidx[i]]; deflated r -> unit entry.
__global__ void __launch_bounds__(DC_T) dc_vectors_kernel(
    int m, const double* __restrict__ sd, const int* __restrict__ perm,
    const int* __restrict__ isnd, const int* __restrict__ ndidx,
    const int* __restrict__ cnt, const double* __restrict__ tau,
    const double* __restrict__ zh, const int64_t* __restrict__ outpos,
    float* __restrict__ W) {
  __shared__ double cd[DC_CH], cz[DC_CH];
  __shared__ int crow[DC_CH];
  const int g = blockIdx.x;
  const int K = cnt[g * 2 + 0];
  const int64_t base = (int64_t)g * m;
  float* Wg = W + (int64_t)g * m * m;
  if (blockIdx.y == 0) {
    for (int r = threadIdx.x; r < m; r += DC_T)
      if (isnd[base + r] < 0)
        Wg[(int64_t)min(max(perm[base + r], 0), m - 1) * m + outpos[base + r]] = 1.f;
  }
  if ((int)(blockIdx.y * DC_T) >= K) return;
  const int j = blockIdx.y * DC_T + threadIdx.x;
  const bool act = j < K;
  double dorg = 0.0, tj = 0.0;
  int64_t col = 0;
  if (act) {
    tj = tau[base + j];
    dorg = sd[base + ndidx[base + ((tj > 0.0 || j == K - 1) ? j : j + 1)]];
    col = outpos[base + ndidx[base + j]];
  }
  double ss = 0.0;
  for (int pass = 0; pass < 2; ++pass) {
    const double inv = pass ? 1.0 / sqrt(ss) : 0.0;
    for (int c0 = 0; c0 < K; c0 += DC_CH) {
      const int len = min(DC_CH, K - c0);
      __syncthreads();
      for (int q = threadIdx.x; q < len; q += DC_T) {
        const int idx = ndidx[base + c0 + q];
        cd[q] = sd[base + idx];
        cz[q] = zh[base + c0 + q];
        crow[q] = min(max(perm[base + idx], 0), m - 1);
      }
      __syncthreads();
      if (!act) continue;
      if (pass == 0) {
        for (int q = 0; q < len; ++q) {
          const double u = cz[q] / ((cd[q] - dorg) - tj);
          ss += u * u;
        }
      } else {
        for (int q = 0; q < len; ++q) {
          const double u = cz[q] / ((cd[q] - dorg) - tj);
          Wg[(int64_t)crow[q] * m + col] = (float)(u * inv);
        }
      }
    }
  }
}

// grid: (G, ceil(m / DC_T)), one thread per column of W: the deflation
// rotations in reverse order on rows (perm[p], perm[i]).
__global__ void __launch_bounds__(DC_T) dc_rotate_kernel(
    int m, const int* __restrict__ perm, const int* __restrict__ cnt,
    const int* __restrict__ rot_idx, const double* __restrict__ rot_cs,
    float* __restrict__ W) {
  const int g = blockIdx.x;
  const int nrot = cnt[g * 2 + 1];
  if (nrot == 0) return;
  const int c = blockIdx.y * DC_T + threadIdx.x;
  if (c >= m) return;
  const int64_t base = (int64_t)g * m;
  float* Wg = W + (int64_t)g * m * m;
  for (int r = nrot - 1; r >= 0; --r) {
    const int a = min(max(perm[base + rot_idx[(base + r) * 2 + 0]], 0), m - 1);
    const int b = min(max(perm[base + rot_idx[(base + r) * 2 + 1]], 0), m - 1);
    const double cc = rot_cs[(base + r) * 2 + 0], s = rot_cs[(base + r) * 2 + 1];
    const double wa = Wg[(int64_t)a * m + c], wb = Wg[(int64_t)b * m + c];
    Wg[(int64_t)a * m + c] = (float)(cc * wa - s * wb);
    Wg[(int64_t)b * m + c] = (float)(s * wa + cc * wb);
  }
}

}  // namespace

int dc_leaf_max() { return 64; }
int dc_max_m() { return 8192; }

void dc_leaves(const float* d_pad, const float* e_pad, int batch, int n_pad, int leaf,
               float* out, hipStream_t s) {
  const int blocks = batch * (n_pad / leaf);
  if (blocks > 0)
    hipLaunchKernelGGL(dc_leaves_kernel, dim3(blocks), dim3(64), 0, s, d_pad, e_pad, n_pad,
                       leaf, out);
}

void dc_merge_front(const double* Dprev, const float* Qprev, const float* e_pad, int n_pad,
                    int h, int S, int G, double* sd, double* sz, int* perm, double* scal,
                    int* isnd, int* ndidx, int* rot_idx, double* rot_cs, int* cnt,
                    double* tau, double* zh, double* vals, hipStream_t s) {
  const int m = 2 * h;
  const size_t lds = (size_t)m * sizeof(double);
  static bool attr = false;
  if (!attr) {
    KFAC_HIP_CHECK(hipFuncSetAttribute((const void*)dc_sort_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       8192 * (int)sizeof(double)));
    attr = true;
  }
  hipLaunchKernelGGL(dc_sort_kernel, dim3(G), dim3(DC_T), lds, s, Dprev, Qprev, e_pad, n_pad,
                     h, S, sd, sz, perm, scal);
  hipLaunchKernelGGL(dc_deflate_kernel, dim3(G), dim3(DC_T), 0, s, m, sd, sz, scal, isnd,
                     ndidx, rot_idx, rot_cs, cnt, vals);
  const dim3 grid(G, (unsigned)ceil_div(m, DC_T));
  hipLaunchKernelGGL(dc_secular_kernel, grid, dim3(DC_T), 0, s, m, sd, sz, ndidx, cnt, scal,
                     tau, vals);
  hipLaunchKernelGGL(dc_zhat_kernel, grid, dim3(DC_T), 0, s, m, sd, sz, ndidx, cnt, scal, tau,
                     zh);
}

void dc_merge_back(int h, int G, const double* sd, const int* perm, const int* isnd,
                   const int* ndidx, const int* cnt, const double* tau, const double* zh,
                   const int64_t* outpos, const int* rot_idx, const double* rot_cs, float* W,
                   hipStream_t s) {
  const int m = 2 * h;
  const dim3 grid(G, (unsigned)ceil_div(m, DC_T));
  hipLaunchKernelGGL(dc_vectors_kernel, grid, dim3(DC_T), 0, s, m, sd, perm, isnd, ndidx, cnt,
                     tau, zh, outpos, W);
  hipLaunchKernelGGL(dc_rotate_kernel, grid, dim3(DC_T), 0, s, m, perm, cnt, rot_idx, rot_cs,
                     W);
}

}  // namespace kfac
