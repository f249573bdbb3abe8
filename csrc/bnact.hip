// Fused training-mode BatchNorm2d (+ residual add) (+ ReLU) for NHWC bf16
// or fp32 activations, forward and backward, for the ResNet models.
//
// Why: in a ResNet-50 step at batch 32 on MI355X the BatchNorm family is
// the largest non-conv cost: MIOpen's 3 forward + 3 backward BN kernels,
// ~2 MIOpen tensor-op kernels, a separate ReLU forward and backward, the
// residual add and the num_batches_tracked increment come to ~4.7 ms of a
// 9.3 ms busy step (profiles/rocprof_steady_sgd_r1_final.txt) for what is
// a few memory passes over each activation.  Here one BN layer is
//   forward : stats partials -> finalize (running stats, counter, scale /
//             shift) -> apply (x*scale + shift [+ residual], ReLU, bf16)
//   backward: partials of dz = dy*(y > 0) and dz*(x - mean) -> finalize
//             (dgamma, dbeta, dx coefficients) -> apply (dx [, d residual])
// All passes move 8 channels per thread per access (one 16-B load of bf16,
// two of fp32), rows are [N*H*W, C] with C % 8 == 0.  Statistics accumulate in fp32 per workgroup
// and in fp64 across workgroups (E[x^2] - E[x]^2 in fp64 does not cancel).
// Semantics follow torch.nn.functional.batch_norm (training=True): biased
// variance to normalise, unbiased variance into running_var, momentum
// update, num_batches_tracked += 1.
#include "common.h"

#include <cstdlib>
#include <cstring>

namespace kfac {

namespace {

constexpr int BN_T = 256;
constexpr int BN_FIN_T = 512;  // finalize block: CH channels x BN_FIN_T / CH lanes

typedef unsigned short us8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void load8(const uint16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ void store8(uint16_t* p, const float* v) {
  uint4 u;
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = (uint32_t)f32_to_bf16_bits(v[2 * i]) |
           ((uint32_t)f32_to_bf16_bits(v[2 * i + 1]) << 16);
  u.x = w[0];
  u.y = w[1];
  u.z = w[2];
  u.w = w[3];
  *reinterpret_cast<uint4*>(p) = u;
}

// fp32 activations: 8 channels = two 16-B accesses
__device__ __forceinline__ void load8(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

__device__ __forceinline__ void store8(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// Raw 8-channel loads: the guarded load loops of the kernels below issue
// only these (no conversion inside the bounds branch), and convert in a
// separate pass.  With the bf16 -> fp32 conversion inside the branch the
// compiler waited for each row's load before issuing the next row's
// (12 `s_waitcnt vmcnt(0)` for 14 loads in the bf16 apply kernel: one
// memory round trip per row instead of one per loop iteration).
template <typename E> struct Raw8 { uint4 w; };
template <> struct Raw8<float> { float4 a, b; };

__device__ __forceinline__ void ldraw8(const uint16_t* p, Raw8<uint16_t>& r) {
  r.w = *reinterpret_cast<const uint4*>(p);
}
__device__ __forceinline__ void ldraw8(const float* p, Raw8<float>& r) {
  r.a = *reinterpret_cast<const float4*>(p);
  r.b = *reinterpret_cast<const float4*>(p + 4);
}
__device__ __forceinline__ void cvt8(const Raw8<uint16_t>& r, float* v) {
  const uint32_t w[4] = {r.w.x, r.w.y, r.w.z, r.w.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void cvt8(const Raw8<float>& r, float* v) {
  v[0] = r.a.x; v[1] = r.a.y; v[2] = r.a.z; v[3] = r.a.w;
  v[4] = r.b.x; v[5] = r.b.y; v[6] = r.b.z; v[7] = r.b.w;
}

// Per-block channel partial sums.  mode 0 (forward): s0 = sum x,
// s1 = sum x^2.  mode 1 (backward): dz = dy * (y > 0 | !relu),
// s0 = sum dz, s1 = sum dz * (x - mean).
template <typename E, int MODE>
__global__ void __launch_bounds__(BN_T) bn_partial_kernel(
    const E* __restrict__ x, const E* __restrict__ dy,
    const E* __restrict__ y, const float* __restrict__ mean, int relu,
    int64_t M, int C, int64_t rows_per_block, float* __restrict__ part) {
  extern __shared__ float sh[];  // [2][RPI][C]
  const int tpr = C / 8;
  const int rpi = BN_T / tpr;
  const int cg = threadIdx.x % tpr, rs = threadIdx.x / tpr;
  const int c0 = cg * 8;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  int64_t r1 = r0 + rows_per_block;
  if (r1 > M) r1 = M;
  float s0[8] = {}, s1[8] = {};
  float mu[8] = {}, msc[8] = {}, msf[8] = {};
  // y == nullptr: the ReLU mask from x (scale / shift follow the mean in
  // the statistics, the forward's fma recomputed bit for bit)
  const bool rec = MODE == 1 && relu && y == nullptr;
  if (MODE == 1 && rs < rpi) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      mu[i] = mean[c0 + i];
      if (rec) {
        msc[i] = mean[2 * C + c0 + i];
        msf[i] = mean[3 * C + c0 + i];
      }
    }
  }
  if (rs < rpi) {
    // U rows per iteration with independent loads: keeps enough 16-B loads
    // in flight per thread to stream at HBM rate from ~400 workgroups
    constexpr int U = MODE == 0 ? 8 : 4;
    for (int64_t rb = r0 + rs; rb < r1; rb += U * (int64_t)rpi) {
      float a[U][8], g[U][8], o[U][8];
      Raw8<E> ra[U], rg[U], ro[U];
      bool ok[U];
      int64_t offs[U];
      // unguarded loads at clamped rows (ok[] masks the sums): guards around
      // the loads made the compiler wait for each row before the next
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = rb + (int64_t)u * rpi;
        ok[u] = r < r1;
        offs[u] = (ok[u] ? r : r1 - 1) * C + c0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ldraw8(x + offs[u], ra[u]);
        if (MODE == 1) ldraw8(dy + offs[u], rg[u]);
      }
      if (MODE == 1 && relu && !rec) {
#pragma unroll
        for (int u = 0; u < U; ++u) ldraw8(y + offs[u], ro[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        cvt8(ra[u], a[u]);
        if (MODE == 1) {
          cvt8(rg[u], g[u]);
          if (relu && !rec) cvt8(ro[u], o[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        if (MODE == 0) {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            s0[i] += a[u][i];
            s1[i] += a[u][i] * a[u][i];
          }
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const bool on = !relu || (rec ? __builtin_fmaf(a[u][i], msc[i], msf[i]) > 0.f
                                                : o[u][i] > 0.f);
            const float gi = on ? g[u][i] : 0.f;
            s0[i] += gi;
            s1[i] += gi * (a[u][i] - mu[i]);
          }
        }
      }
    }
  }
  float* sh0 = sh;
  float* sh1 = sh + rpi * C;
  if (rs < rpi) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sh0[rs * C + c0 + i] = s0[i];
      sh1[rs * C + c0 + i] = s1[i];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += BN_T) {
    float a = 0.f, b = 0.f;
    for (int q = 0; q < rpi; ++q) {
      a += sh0[q * C + c];
      b += sh1[q * C + c];
    }
    part[((int64_t)blockIdx.x * 2) * C + c] = a;
    part[((int64_t)blockIdx.x * 2 + 1) * C + c] = b;
  }
}

// fp64 reduction of the partials: CH channels x (BN_FIN_T / CH) lanes per
// block.  CH = 32 when there are few partial blocks; with many (a
// convolution epilogue's partials: one per 64 output rows, 1568 for a
// 56x56 layer at batch 32) fewer channels and more lanes per block, so each
// lane walks fewer latency-bound loads (fin_ch_for).  The order is fixed for
// a given (nblk, C): deterministic.
template <int CH>
__device__ __forceinline__ void reduce_parts(const float* __restrict__ part, int nblk, int C,
                                             int c, double& a, double& b) {
  constexpr int L = BN_FIN_T / CH;
  __shared__ double ra[L][CH], rb[L][CH];
  const int lane = threadIdx.x / CH, cl = threadIdx.x % CH;
  double sa = 0.0, sb = 0.0;
  if (c < C) {
    // 4 independent loads in flight per step (the finalize is latency bound)
    int blk = lane;
    for (; blk + 3 * L < nblk; blk += 4 * L) {
      float va[4], vb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        va[u] = part[((int64_t)(blk + u * L) * 2) * C + c];
        vb[u] = part[((int64_t)(blk + u * L) * 2 + 1) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        sa += (double)va[u];
        sb += (double)vb[u];
      }
    }
    for (; blk < nblk; blk += L) {
      sa += (double)part[((int64_t)blk * 2) * C + c];
      sb += (double)part[((int64_t)blk * 2 + 1) * C + c];
    }
  }
  ra[lane][cl] = sa;
  rb[lane][cl] = sb;
  __syncthreads();
  a = 0.0;
  b = 0.0;
  if (threadIdx.x < CH) {
    for (int q = 0; q < L; ++q) {
      a += ra[q][cl];
      b += rb[q][cl];
    }
  }
}

// stats[4][C]: mean, invstd, scale, shift
template <int CH>
__global__ void __launch_bounds__(BN_FIN_T) bn_fwd_finalize_kernel(
    const float* __restrict__ part, int nblk, int64_t M, int C,
    const float* __restrict__ weight, const float* __restrict__ bias,
    float* __restrict__ running_mean, float* __restrict__ running_var,
    int64_t* __restrict__ num_batches, float momentum, float eps,
    float* __restrict__ stats) {
  const int c = blockIdx.x * CH + threadIdx.x % CH;
  double s, q;
  reduce_parts<CH>(part, nblk, C, c, s, q);
  if (threadIdx.x >= CH || c >= C) return;
  const double mean = s / (double)M;
  double var = q / (double)M - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float w = weight ? weight[c] : 1.f;
  const float b = bias ? bias[c] : 0.f;
  const float scale = w * invstd;
  stats[c] = (float)mean;
  stats[C + c] = invstd;
  stats[2 * C + c] = scale;
  stats[3 * C + c] = b - (float)mean * scale;
  if (running_mean) {
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
    const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unb;
  }
  if (num_batches && c == 0) num_batches[0] += 1;
}

// Apply passes: each thread owns one 8-channel group for the whole launch
// (per-channel constants in registers, no index division) and streams 4
// rows per iteration with independent 16-B loads.
template <typename E>
__global__ void __launch_bounds__(BN_T) bn_fwd_apply_kernel(
    const E* __restrict__ x, const E* __restrict__ res,
    const float* __restrict__ stats, int relu, int64_t M, int C,
    E* __restrict__ y) {
  const int tpr = C / 8;
  const int rpi = BN_T / tpr;
  const int cg = threadIdx.x % tpr, rs = threadIdx.x / tpr;
  if (rs >= rpi) return;
  const int c0 = cg * 8;
  float sc[8], sf[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = stats[2 * C + c0 + i];
    sf[i] = stats[3 * C + c0 + i];
  }
  const int64_t step = (int64_t)gridDim.x * 4 * rpi;
  for (int64_t rb = (int64_t)blockIdx.x * 4 * rpi + rs; rb < M; rb += step) {
    float a[4][8], r[4][8];
    Raw8<E> ra[4], rr[4];
    // unguarded loads at clamped rows (masked at the store): per-row
    // guards around the loads made the compiler wait for each row's data
    // before issuing the next row's loads
    int64_t offs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t row = rb + (int64_t)u * rpi;
      offs[u] = (row < M ? row : M - 1) * C + c0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) ldraw8(x + offs[u], ra[u]);
    if (res) {
#pragma unroll
      for (int u = 0; u < 4; ++u) ldraw8(res + offs[u], rr[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (rb + (int64_t)u * rpi >= M) continue;
      cvt8(ra[u], a[u]);
      if (res) cvt8(rr[u], r[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t row = rb + (int64_t)u * rpi;
      if (row >= M) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float o = __builtin_fmaf(a[u][i], sc[i], sf[i]);
        if (res) o += r[u][i];
        a[u][i] = relu ? fmaxf(o, 0.f) : o;
      }
      store8(y + row * C + c0, a[u]);
    }
  }
}

// coef[3][C]: k1, k2, k3 with dx = k1*dz + k2 + k3*(x - mean)
template <int CH>
__global__ void __launch_bounds__(BN_FIN_T) bn_bwd_finalize_kernel(
    const float* __restrict__ part, int nblk, int64_t M, int C,
    const float* __restrict__ weight, const float* __restrict__ stats,
    float* __restrict__ dweight, float* __restrict__ dbias, float* __restrict__ coef) {
  const int c = blockIdx.x * CH + threadIdx.x % CH;
  double sdz, sdzx;
  reduce_parts<CH>(part, nblk, C, c, sdz, sdzx);
  if (threadIdx.x >= CH || c >= C) return;
  const double invstd = stats[C + c];
  const double w = weight ? weight[c] : 1.0;
  if (dweight) dweight[c] = (float)(sdzx * invstd);
  if (dbias) dbias[c] = (float)sdz;
  const double k1 = w * invstd;
  coef[c] = (float)k1;
  coef[C + c] = (float)(-k1 * sdz / (double)M);
  coef[2 * C + c] = (float)(-k1 * invstd * invstd * sdzx / (double)M);
}

template <typename E>
__global__ void __launch_bounds__(BN_T) bn_bwd_apply_kernel(
    const E* __restrict__ x, const E* __restrict__ dy,
    const E* __restrict__ y, const float* __restrict__ stats,
    const float* __restrict__ coef, int relu, int64_t M, int C,
    E* __restrict__ dx, E* __restrict__ dres) {
  const int tpr = C / 8;
  const int rpi = BN_T / tpr;
  const int cg = threadIdx.x % tpr, rs = threadIdx.x / tpr;
  if (rs >= rpi) return;
  const int c0 = cg * 8;
  float mu[8], k1[8], k2[8], k3[8], msc[8], msf[8];
  const bool rec = relu && y == nullptr;  // ReLU mask from x (bn_partial_kernel)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mu[i] = stats[c0 + i];
    msc[i] = stats[2 * C + c0 + i];
    msf[i] = stats[3 * C + c0 + i];
    k1[i] = coef[c0 + i];
    k2[i] = coef[C + c0 + i];
    k3[i] = coef[2 * C + c0 + i];
  }
  const int64_t step = (int64_t)gridDim.x * 4 * rpi;
  for (int64_t rb = (int64_t)blockIdx.x * 4 * rpi + rs; rb < M; rb += step) {
    float a[4][8], g[4][8], o[4][8];
    Raw8<E> ra[4], rg[4], ro[4];
    // unguarded loads at clamped rows (masked at the store), as forward
    int64_t offs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t row = rb + (int64_t)u * rpi;
      offs[u] = (row < M ? row : M - 1) * C + c0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      ldraw8(x + offs[u], ra[u]);
      ldraw8(dy + offs[u], rg[u]);
    }
    if (relu && !rec) {
#pragma unroll
      for (int u = 0; u < 4; ++u) ldraw8(y + offs[u], ro[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (rb + (int64_t)u * rpi >= M) continue;
      cvt8(ra[u], a[u]);
      cvt8(rg[u], g[u]);
      if (relu && !rec) cvt8(ro[u], o[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t row = rb + (int64_t)u * rpi;
      if (row >= M) continue;
      const int64_t off = row * C + c0;
      if (rec) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
          g[u][i] = __builtin_fmaf(a[u][i], msc[i], msf[i]) > 0.f ? g[u][i] : 0.f;
      } else if (relu) {
#pragma unroll
        for (int i = 0; i < 8; ++i) g[u][i] = o[u][i] > 0.f ? g[u][i] : 0.f;
      }
      if (dres) store8(dres + off, g[u]);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[u][i] = k1[i] * g[u][i] + k2[i] + k3[i] * (a[u][i] - mu[i]);
      store8(dx + off, a[u]);
    }
  }
}

// ---- small-activation path (ResNet stages 2-4): two launches per
// direction instead of three.  Partial sums are taken per (channel slice,
// row chunk) block with few row chunks, so every apply block can reduce the
// partials of its own channel slice (P x 64 x 2 floats) and finalise those
// channels itself; the separate finalize launch -- ~5 us of fixed cost per
// BN layer and direction on MI355X -- disappears.  Blocks in row chunk 0
// publish the statistics (forward) or dweight / dbias (backward).
constexpr int SB_CW = 64;    // channels per slice
constexpr int SB_PMAX = 64;  // row chunks of the partial pass

__device__ __host__ __forceinline__ int sliced_cw(int C) { return C < SB_CW ? C : SB_CW; }

template <typename E, int MODE>
__global__ void __launch_bounds__(BN_T) bn_partial_sliced_kernel(
    const E* __restrict__ x, const E* __restrict__ dy,
    const E* __restrict__ y, const float* __restrict__ mean, int relu,
    int64_t M, int C, int64_t rows_per_chunk, float* __restrict__ part) {
  __shared__ float sh[2][BN_T * 8];  // [RT][cw] per statistic
  const int cw = sliced_cw(C);
  const int tpc = cw / 8, RT = BN_T / tpc;
  const int tc = threadIdx.x % tpc, rt = threadIdx.x / tpc;
  const int c0 = blockIdx.x * cw + tc * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = r0 + rows_per_chunk < M ? r0 + rows_per_chunk : M;
  float s0[8] = {}, s1[8] = {}, mu[8] = {}, msc[8] = {}, msf[8] = {};
  // y == nullptr: the ReLU mask from x (as bn_partial_kernel)
  const bool rec = MODE == 1 && relu && y == nullptr;
  if (MODE == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      mu[i] = mean[c0 + i];
      if (rec) {
        msc[i] = mean[2 * C + c0 + i];
        msf[i] = mean[3 * C + c0 + i];
      }
    }
  }
  constexpr int U = 4;
  for (int64_t rb = r0 + rt; rb < r1; rb += U * (int64_t)RT) {
    float a[U][8], g[U][8], o[U][8];
    Raw8<E> ra[U], rg[U], ro[U];
    bool ok[U];
    int64_t offs[U];
    // unguarded loads at clamped rows (ok[] masks the sums): guards around
    // the loads made the compiler wait for each row before the next
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = rb + (int64_t)u * RT;
      ok[u] = r < r1;
      offs[u] = (ok[u] ? r : r1 - 1) * C + c0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ldraw8(x + offs[u], ra[u]);
      if (MODE == 1) ldraw8(dy + offs[u], rg[u]);
    }
    if (MODE == 1 && relu && !rec) {
#pragma unroll
      for (int u = 0; u < U; ++u) ldraw8(y + offs[u], ro[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      cvt8(ra[u], a[u]);
      if (MODE == 1) {
        cvt8(rg[u], g[u]);
        if (relu && !rec) cvt8(ro[u], o[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (MODE == 0) {
          s0[i] += a[u][i];
          s1[i] += a[u][i] * a[u][i];
        } else {
          const bool on = !relu || (rec ? __builtin_fmaf(a[u][i], msc[i], msf[i]) > 0.f
                                                : o[u][i] > 0.f);
            const float gi = on ? g[u][i] : 0.f;
          s0[i] += gi;
          s1[i] += gi * (a[u][i] - mu[i]);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sh[0][rt * cw + tc * 8 + i] = s0[i];
    sh[1][rt * cw + tc * 8 + i] = s1[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < cw; c += BN_T) {
    float a = 0.f, b = 0.f;
    for (int q = 0; q < RT; ++q) {
      a += sh[0][q * cw + c];
      b += sh[1][q * cw + c];
    }
    const int ch = blockIdx.x * cw + c;
    part[((int64_t)blockIdx.y * 2) * C + ch] = a;
    part[((int64_t)blockIdx.y * 2 + 1) * C + ch] = b;
  }
}

// fp64 sums of the P partials of this block's channel slice -> tot[2][cw]
__device__ __forceinline__ void sliced_reduce(const float* __restrict__ part, int P, int C, int cw,
                                              double (*tot)[SB_CW]) {
  __shared__ double ra[BN_T], rb[BN_T];
  const int nsub = BN_T / cw;
  const int ch = threadIdx.x % cw, sub = threadIdx.x / cw;
  const int c = blockIdx.x * cw + ch;
  double sa = 0.0, sb = 0.0;
  for (int p = sub; p < P; p += nsub) {
    sa += (double)part[((int64_t)p * 2) * C + c];
    sb += (double)part[((int64_t)p * 2 + 1) * C + c];
  }
  ra[threadIdx.x] = sa;
  rb[threadIdx.x] = sb;
  __syncthreads();
  if ((int)threadIdx.x < cw) {
    double a = 0.0, b = 0.0;
    for (int q = 0; q < nsub; ++q) {
      a += ra[q * cw + threadIdx.x];
      b += rb[q * cw + threadIdx.x];
    }
    tot[0][threadIdx.x] = a;
    tot[1][threadIdx.x] = b;
  }
}

// forward: finalise this slice's channels, then x*scale + shift (+ res) (ReLU)
template <typename E>
__global__ void __launch_bounds__(BN_T) bn_fwd_apply_sliced_kernel(
    const E* __restrict__ x, const E* __restrict__ res,
    const float* __restrict__ part, int P, int64_t M, int C, int64_t rows_per_chunk,
    const float* __restrict__ weight, const float* __restrict__ bias,
    float* __restrict__ running_mean, float* __restrict__ running_var,
    int64_t* __restrict__ num_batches, float momentum, float eps, int relu,
    float* __restrict__ stats, E* __restrict__ y) {
  __shared__ double tot[2][SB_CW];
  __shared__ float ssc[SB_CW], ssf[SB_CW];
  const int cw = sliced_cw(C);
  sliced_reduce(part, P, C, cw, tot);
  __syncthreads();
  if ((int)threadIdx.x < cw) {
    const int c = blockIdx.x * cw + threadIdx.x;
    const double mean = tot[0][threadIdx.x] / (double)M;
    double var = tot[1][threadIdx.x] / (double)M - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float w = weight ? weight[c] : 1.f;
    const float b = bias ? bias[c] : 0.f;
    const float scale = w * invstd;
    const float shift = b - (float)mean * scale;
    ssc[threadIdx.x] = scale;
    ssf[threadIdx.x] = shift;
    if (blockIdx.y == 0) {
      stats[c] = (float)mean;
      stats[C + c] = invstd;
      stats[2 * C + c] = scale;
      stats[3 * C + c] = shift;
      if (running_mean) {
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
        const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unb;
      }
      if (num_batches && c == 0) num_batches[0] += 1;
    }
  }
  __syncthreads();
  const int tpc = cw / 8, RT = BN_T / tpc;
  const int tc = threadIdx.x % tpc, rt = threadIdx.x / tpc;
  const int c0 = blockIdx.x * cw + tc * 8;
  float sc[8], sf[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = ssc[tc * 8 + i];
    sf[i] = ssf[tc * 8 + i];
  }
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = r0 + rows_per_chunk < M ? r0 + rows_per_chunk : M;
  for (int64_t rb = r0 + rt; rb < r1; rb += 4 * (int64_t)RT) {
    float a[4][8], r[4][8];
    Raw8<E> ra[4], rr[4];
    // unguarded loads at clamped rows (masked at the store): per-row
    // guards around the loads made the compiler wait for each row's data
    // before issuing the next row's loads
    int64_t offs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t row = rb + (int64_t)u * RT;
      offs[u] = (row < r1 ? row : r1 - 1) * C + c0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) ldraw8(x + offs[u], ra[u]);
    if (res) {
#pragma unroll
      for (int u = 0; u < 4; ++u) ldraw8(res + offs[u], rr[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (rb + (int64_t)u * RT >= r1) continue;
      cvt8(ra[u], a[u]);
      if (res) cvt8(rr[u], r[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t row = rb + (int64_t)u * RT;
      if (row >= r1) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float o = __builtin_fmaf(a[u][i], sc[i], sf[i]);
        if (res) o += r[u][i];
        a[u][i] = relu ? fmaxf(o, 0.f) : o;
      }
      store8(y + row * C + c0, a[u]);
    }
  }
}

// backward: finalise dweight / dbias and the dx coefficients of this slice,
// then dx = k1*dz + k2 + k3*(x - mean) (and d residual = dz)
template <typename E>
__global__ void __launch_bounds__(BN_T) bn_bwd_apply_sliced_kernel(
    const E* __restrict__ x, const E* __restrict__ dy,
    const E* __restrict__ y, const float* __restrict__ part, int P, int64_t M, int C,
    int64_t rows_per_chunk, const float* __restrict__ weight, const float* __restrict__ stats,
    float* __restrict__ dweight, float* __restrict__ dbias, int relu,
    E* __restrict__ dx, E* __restrict__ dres) {
  __shared__ double tot[2][SB_CW];
  __shared__ float sk1[SB_CW], sk2[SB_CW], sk3[SB_CW], smu[SB_CW];
  const int cw = sliced_cw(C);
  sliced_reduce(part, P, C, cw, tot);
  __syncthreads();
  if ((int)threadIdx.x < cw) {
    const int c = blockIdx.x * cw + threadIdx.x;
    const double sdz = tot[0][threadIdx.x], sdzx = tot[1][threadIdx.x];
    const double invstd = stats[C + c];
    const double w = weight ? weight[c] : 1.0;
    if (blockIdx.y == 0) {
      if (dweight) dweight[c] = (float)(sdzx * invstd);
      if (dbias) dbias[c] = (float)sdz;
    }
    const double k1 = w * invstd;
    sk1[threadIdx.x] = (float)k1;
    sk2[threadIdx.x] = (float)(-k1 * sdz / (double)M);
    sk3[threadIdx.x] = (float)(-k1 * invstd * invstd * sdzx / (double)M);
    smu[threadIdx.x] = stats[c];
  }
  __syncthreads();
  const int tpc = cw / 8, RT = BN_T / tpc;
  const int tc = threadIdx.x % tpc, rt = threadIdx.x / tpc;
  const int c0 = blockIdx.x * cw + tc * 8;
  float mu[8], k1[8], k2[8], k3[8], msc[8], msf[8];
  const bool rec = relu && y == nullptr;  // ReLU mask from x (bn_partial_kernel)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mu[i] = smu[tc * 8 + i];
    msc[i] = stats[2 * C + c0 + i];
    msf[i] = stats[3 * C + c0 + i];
    k1[i] = sk1[tc * 8 + i];
    k2[i] = sk2[tc * 8 + i];
    k3[i] = sk3[tc * 8 + i];
  }
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = r0 + rows_per_chunk < M ? r0 + rows_per_chunk : M;
  for (int64_t rb = r0 + rt; rb < r1; rb += 4 * (int64_t)RT) {
    float a[4][8], g[4][8], o[4][8];
    Raw8<E> ra[4], rg[4], ro[4];
    // unguarded loads at clamped rows (masked at the store), as forward
    int64_t offs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t row = rb + (int64_t)u * RT;
      offs[u] = (row < r1 ? row : r1 - 1) * C + c0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      ldraw8(x + offs[u], ra[u]);
      ldraw8(dy + offs[u], rg[u]);
    }
    if (relu && !rec) {
#pragma unroll
      for (int u = 0; u < 4; ++u) ldraw8(y + offs[u], ro[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (rb + (int64_t)u * RT >= r1) continue;
      cvt8(ra[u], a[u]);
      cvt8(rg[u], g[u]);
      if (relu && !rec) cvt8(ro[u], o[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t row = rb + (int64_t)u * RT;
      if (row >= r1) continue;
      const int64_t off = row * C + c0;
      if (rec) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
          g[u][i] = __builtin_fmaf(a[u][i], msc[i], msf[i]) > 0.f ? g[u][i] : 0.f;
      } else if (relu) {
#pragma unroll
        for (int i = 0; i < 8; ++i) g[u][i] = o[u][i] > 0.f ? g[u][i] : 0.f;
      }
      if (dres) store8(dres + off, g[u]);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[u][i] = k1[i] * g[u][i] + k2[i] + k3[i] * (a[u][i] - mu[i]);
      store8(dx + off, a[u]);
    }
  }
}

// (partial chunks, apply chunks, rows per partial chunk, rows per apply
// chunk) of the sliced path, or false when the activation is large enough
// for the three-launch path (whose ~400 partial blocks keep HBM busy)
bool sliced_plan(int64_t M, int C, int* P, int* Q, int64_t* rp, int64_t* rq) {
  // KFAC_BN_SLICED=0: always the three-launch path (A/B runs)
  static const bool enabled = [] {
    const char* e = std::getenv("KFAC_BN_SLICED");
    return e == nullptr || std::strcmp(e, "0") != 0;
  }();
  if (!enabled) return false;
  // channel slices of 8 * 2^k channels (whole thread columns per block)
  if (C > SB_CW ? C % SB_CW != 0 : (C != 8 && C != 16 && C != 32 && C != 64)) return false;
  const int cw = sliced_cw(C);
  const int nsl = C / cw;
  const int rt = BN_T / (cw / 8);
  int p = (int)ceil_div(256, nsl);
  if (p > SB_PMAX) p = SB_PMAX;
  if (p < 1) p = 1;
  const int64_t rows = ceil_div(M, (int64_t)p);
  // > 32 rows per thread, or too few partial blocks to stream the tensor:
  // the three-launch path
  if (rows > 32 * (int64_t)rt || (int64_t)nsl * ceil_div(M, rows) < 128) return false;
  int q = (int)ceil_div(512, nsl);
  const int64_t qmax = ceil_div(M, 4 * (int64_t)rt);  // >= one unrolled pass per thread
  if (q > qmax) q = (int)qmax;
  if (q < 1) q = 1;
  *P = (int)ceil_div(M, rows);
  *rp = rows;
  *rq = ceil_div(M, (int64_t)q);
  *Q = (int)ceil_div(M, *rq);
  return true;
}

int apply_grid(int64_t M, int C) {
  const int rpi = BN_T / (C / 8);
  int64_t g = ceil_div(M, 4 * (int64_t)rpi);
  return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

}  // namespace

// rows per partial block and block count for [M, C]
void bn_partition(int64_t M, int C, int64_t* rows_per_block, int* nblk) {
  int P, Q;
  int64_t rp, rq;
  if (sliced_plan(M, C, &P, &Q, &rp, &rq)) {
    *rows_per_block = rp;
    *nblk = P;
    return;
  }
  // ~400 workgroups on the big activations (8 / 4 rows of loads in flight
  // per thread keep HBM busy; few partials keep the finalize short), at
  // least 32 rows and one full unrolled iteration per workgroup
  const int rpi = BN_T / (C / 8);
  int64_t r = ceil_div(M, 400);
  if (r < (int64_t)rpi * 8) r = (int64_t)rpi * 8;
  if (r < 32) r = 32;
  *rows_per_block = r;
  *nblk = (int)ceil_div(M, r);
}

int bn_max_c() { return 8 * BN_T; }

namespace {

// channels per finalize block: enough lanes that each walks <= ~16 of the
// nblk partial rows (KFAC_BN_FIN_CH=32 pins the old 32 x 16 layout)
int fin_ch_for(int nblk) {
  static const int pin = [] {
    const char* e = std::getenv("KFAC_BN_FIN_CH");
    return e != nullptr ? std::atoi(e) : 0;
  }();
  if (pin == 4 || pin == 8 || pin == 16 || pin == 32) return pin;
  int lanes = 16;
  while (lanes < BN_FIN_T / 4 && lanes * 16 < nblk) lanes *= 2;
  return BN_FIN_T / lanes;
}

void launch_fwd_finalize(const float* part, int nblk, int64_t M, int C, const float* weight,
                         const float* bias, float* running_mean, float* running_var,
                         int64_t* num_batches, float momentum, float eps, float* stats,
                         hipStream_t s) {
  const int ch = fin_ch_for(nblk);
#define KFAC_FWD_FIN(CHV)                                                                     \
  hipLaunchKernelGGL(bn_fwd_finalize_kernel<CHV>, dim3((unsigned)ceil_div(C, CHV)),            \
                     dim3(BN_FIN_T), 0, s, part, nblk, M, C, weight, bias, running_mean,       \
                     running_var, num_batches, momentum, eps, stats)
  if (ch == 4) KFAC_FWD_FIN(4);
  else if (ch == 8) KFAC_FWD_FIN(8);
  else if (ch == 16) KFAC_FWD_FIN(16);
  else KFAC_FWD_FIN(32);
#undef KFAC_FWD_FIN
}

void launch_bwd_finalize(const float* part, int nblk, int64_t M, int C, const float* weight,
                         const float* stats, float* dweight, float* dbias, float* coef,
                         hipStream_t s) {
  const int ch = fin_ch_for(nblk);
#define KFAC_BWD_FIN(CHV)                                                                     \
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<CHV>, dim3((unsigned)ceil_div(C, CHV)),            \
                     dim3(BN_FIN_T), 0, s, part, nblk, M, C, weight, stats, dweight, dbias,    \
                     coef)
  if (ch == 4) KFAC_BWD_FIN(4);
  else if (ch == 8) KFAC_BWD_FIN(8);
  else if (ch == 16) KFAC_BWD_FIN(16);
  else KFAC_BWD_FIN(32);
#undef KFAC_BWD_FIN
}

template <typename E>
void bn_forward_t(const E* x, const E* res, const float* weight, const float* bias,
                  float* running_mean, float* running_var, int64_t* num_batches, float momentum,
                  float eps, int relu, int64_t M, int C, float* part, float* stats, E* y,
                  hipStream_t s, const float* ext_part, int ext_p) {
  if (ext_part != nullptr) {
    // statistics partials from the producing convolution's epilogue
    // ([ext_p][2][C]): no pass over x before the apply
    int P, Q;
    int64_t rp, rq;
    if (sliced_plan(M, C, &P, &Q, &rp, &rq) && ext_p <= 2 * SB_PMAX) {
      // small activation: each apply block reduces its slice's partials
      const unsigned nsl = (unsigned)(C / sliced_cw(C));
      hipLaunchKernelGGL(bn_fwd_apply_sliced_kernel<E>, dim3(nsl, (unsigned)Q), dim3(BN_T), 0, s,
                         x, res, ext_part, ext_p, M, C, rq, weight, bias, running_mean,
                         running_var, num_batches, momentum, eps, relu, stats, y);
      return;
    }
    launch_fwd_finalize(ext_part, ext_p, M, C, weight, bias, running_mean, running_var,
                        num_batches, momentum, eps, stats, s);
    hipLaunchKernelGGL(bn_fwd_apply_kernel<E>, dim3(apply_grid(M, C)), dim3(BN_T), 0, s, x, res,
                       stats, relu, M, C, y);
    return;
  }
  {
    int P, Q;
    int64_t rp, rq;
    if (sliced_plan(M, C, &P, &Q, &rp, &rq)) {
      const unsigned nsl = (unsigned)(C / sliced_cw(C));
      hipLaunchKernelGGL((bn_partial_sliced_kernel<E, 0>), dim3(nsl, (unsigned)P), dim3(BN_T), 0,
                         s, x, nullptr, nullptr, nullptr, 0, M, C, rp, part);
      hipLaunchKernelGGL(bn_fwd_apply_sliced_kernel<E>, dim3(nsl, (unsigned)Q), dim3(BN_T), 0, s,
                         x, res, part, P, M, C, rq, weight, bias, running_mean, running_var,
                         num_batches, momentum, eps, relu, stats, y);
      return;
    }
  }
  int64_t rpb;
  int nblk;
  bn_partition(M, C, &rpb, &nblk);
  const int rpi = BN_T / (C / 8);
  const size_t shm = (size_t)2 * rpi * C * sizeof(float);
  hipLaunchKernelGGL((bn_partial_kernel<E, 0>), dim3(nblk), dim3(BN_T), shm, s, x, nullptr,
                     nullptr, nullptr, 0, M, C, rpb, part);
  launch_fwd_finalize(part, nblk, M, C, weight, bias, running_mean, running_var, num_batches,
                      momentum, eps, stats, s);
  hipLaunchKernelGGL(bn_fwd_apply_kernel<E>, dim3(apply_grid(M, C)), dim3(BN_T), 0, s, x, res,
                     stats, relu, M, C, y);
}

template <typename E>
void bn_backward_t(const E* x, const E* dy, const E* y, const float* weight, const float* stats,
                   int relu, int64_t M, int C, float* part, float* coef, float* dweight,
                   float* dbias, E* dx, E* dres, hipStream_t s) {
  // Without a residual the ReLU mask y > 0 is x * scale + shift > 0, which
  // the kernels recompute from the x they read anyway: two passes over y
  // fewer per layer (KFAC_BN_MASK_FROM_Y=1 reads y as before)
  static const bool from_y = [] {
    const char* e = std::getenv("KFAC_BN_MASK_FROM_Y");
    return e != nullptr && std::strcmp(e, "1") == 0;
  }();
  if (dres == nullptr && !from_y) y = nullptr;
  {
    int P, Q;
    int64_t rp, rq;
    if (sliced_plan(M, C, &P, &Q, &rp, &rq)) {
      const unsigned nsl = (unsigned)(C / sliced_cw(C));
      hipLaunchKernelGGL((bn_partial_sliced_kernel<E, 1>), dim3(nsl, (unsigned)P), dim3(BN_T), 0,
                         s, x, dy, y, stats, relu, M, C, rp, part);
      hipLaunchKernelGGL(bn_bwd_apply_sliced_kernel<E>, dim3(nsl, (unsigned)Q), dim3(BN_T), 0, s,
                         x, dy, y, part, P, M, C, rq, weight, stats, dweight, dbias, relu, dx,
                         dres);
      (void)coef;  // the sliced path keeps its coefficients in LDS
      return;
    }
  }
  int64_t rpb;
  int nblk;
  bn_partition(M, C, &rpb, &nblk);
  const int rpi = BN_T / (C / 8);
  const size_t shm = (size_t)2 * rpi * C * sizeof(float);
  hipLaunchKernelGGL((bn_partial_kernel<E, 1>), dim3(nblk), dim3(BN_T), shm, s, x, dy, y, stats,
                     relu, M, C, rpb, part);
  launch_bwd_finalize(part, nblk, M, C, weight, stats, dweight, dbias, coef, s);
  hipLaunchKernelGGL(bn_bwd_apply_kernel<E>, dim3(apply_grid(M, C)), dim3(BN_T), 0, s, x, dy, y,
                     stats, coef, relu, M, C, dx, dres);
}

}  // namespace

// dtype: kBF16 (NHWC bf16, the autocast path) or kF32 (NHWC fp32)
void bn_forward(int dtype, const void* x, const void* res, const float* weight,
                const float* bias, float* running_mean, float* running_var,
                int64_t* num_batches, float momentum, float eps, int relu, int64_t M,
                int C, float* part, float* stats, void* y, hipStream_t s,
                const float* ext_part, int ext_p) {
  if (dtype == kF32)
    bn_forward_t((const float*)x, (const float*)res, weight, bias, running_mean, running_var,
                 num_batches, momentum, eps, relu, M, C, part, stats, (float*)y, s, ext_part,
                 ext_p);
  else
    bn_forward_t((const uint16_t*)x, (const uint16_t*)res, weight, bias, running_mean,
                 running_var, num_batches, momentum, eps, relu, M, C, part, stats,
                 (uint16_t*)y, s, ext_part, ext_p);
}

void bn_backward(int dtype, const void* x, const void* dy, const void* y, const float* weight,
                 const float* stats, int relu, int64_t M, int C, float* part, float* coef,
                 float* dweight, float* dbias, void* dx, void* dres, hipStream_t s) {
  if (dtype == kF32)
    bn_backward_t((const float*)x, (const float*)dy, (const float*)y, weight, stats, relu, M, C,
                  part, coef, dweight, dbias, (float*)dx, (float*)dres, s);
  else
    bn_backward_t((const uint16_t*)x, (const uint16_t*)dy, (const uint16_t*)y, weight, stats,
                  relu, M, C, part, coef, dweight, dbias, (uint16_t*)dx, (uint16_t*)dres, s);
}

}  // namespace kfac
