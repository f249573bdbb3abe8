// K-HIP-3, two-stage eigensolver, stage 2: band (width 16) -> tridiagonal by
// bulge chasing, B = Q2 T Q2^T.
//
// Sweep j (j = 0..n-3) annihilates column j below its subdiagonal with a
// 16-long Householder reflector on rows j+1..j+16 (task 0), then chases the
// bulge that reflector creates down the band: task k >= 1 right-applies the
// previous reflector to the 16 x 16 block below it (rows J1..J2 = j+1+16k ..
// +15, columns j+1+16(k-1) .. +15), annihilates that block's FIRST column
// with a new reflector on rows J1..J2, left-applies it to the block's other
// columns and two-sidedly to the diagonal block [J1..J2]^2.  The rest of each
// bulge stays (bandwidth <= 2*16-2) and is reduced by the next sweeps.
// Every task touches the 32 x 32 window starting at column j+1+16(k-1), so
// task (j, k) only has to follow task (j, k-1) and task (j-1, k+2): sweeps
// run as a pipeline with a lag of three tasks (tools: the float64 oracle in
// distributed_kfac_pytorch_amd/ops/twostage.py replays the schedule and
// matches the sequential order bit for bit).
//
// One 1024-thread workgroup per matrix: wave w runs sweeps w, w+16, ...;
// per-wave progress words in LDS order the pipeline (workgroup-scope
// release / acquire: the waves share the CU's L1; band loads bypass it).
// The band lives in L2-resident global memory, column-major with 32
// distances per column (AB[c][d] = B[c+d][c]); padding columns past n are
// zero so windows never need bounds checks.  A task's operands sit in
// registers, one 16-row block per lane group: lane (r, grp) holds 8 columns
// of row r of the bulge block (grp 0, 1) or of the diagonal block (grp 2, 3).
// Reflectors (v[0] = 1 stored, tau) go to V2[j][k][16] / tau2[j][k] for the
// back-transform (csrc/bt2.hip).
#include "common.h"

namespace kfac {

namespace {

constexpr int S2_B = 16;
constexpr int S2_LD = 2 * S2_B;  // band storage: distances 0..31 per column
constexpr int S2_WAVES = 16;
constexpr int S2_T = 64 * S2_WAVES;
constexpr int S2_SPIN_LIMIT = 1 << 24;  // ~1 s: a correct run waits microseconds

__device__ __forceinline__ int ntasks(int j, int n) { return 1 + (n - 2 - j) / S2_B; }

// sum over the 16 lanes of each DPP row, left in every lane of the row
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_mov<0xb1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_mov<0x4e>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v;
}

__device__ __forceinline__ float rdlane(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

__device__ __forceinline__ float ld_nt(const float* p) { return __builtin_nontemporal_load(p); }

__global__ void __launch_bounds__(S2_T) sb2st_kernel(float* __restrict__ ABall, int64_t sAB,
                                                     int n, float* __restrict__ V2all,
                                                     float* __restrict__ tau2all, int64_t sV2,
                                                     int kmax, float* __restrict__ dout,
                                                     float* __restrict__ eout,
                                                     int* __restrict__ err) {
  const int b = blockIdx.x;
  float* AB = ABall + (int64_t)b * sAB;
  float* V2 = V2all + (int64_t)b * sV2 * S2_B;
  float* tau2s = tau2all + (int64_t)b * sV2;
  __shared__ int prog[S2_WAVES];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int r = l & 15, grp = l >> 4;
  const bool hi = (grp & 1) != 0;
  const bool isD = grp >= 2;
  if (l == 0) prog[w] = (w - S2_WAVES) * 65536 + 0xFFFF;  // "sweep w-16 done"
  __syncthreads();
  bool abort = false;
  const int nsweep = n - 2;

  for (int j = w; j < nsweep && !abort; j += S2_WAVES) {
    const int nk = ntasks(j, n);
    const int nkp = j > 0 ? ntasks(j - 1, n) : 0;
    float vpc[8];  // previous reflector at this lane's 8 columns
#pragma unroll
    for (int i = 0; i < 8; ++i) vpc[i] = 0.f;
    float taup = 0.f;
    for (int k = 0; k < nk; ++k) {
      // ---- wait for task (j-1, min(k+2, nkp-1))
      if (j > 0) {
        const int need = k + 3 < nkp ? k + 3 : 0xFFFF;
        const int target = (j - 1) * 65536 + need;
        int spins = 0;
        while (__hip_atomic_load(&prog[(w + S2_WAVES - 1) % S2_WAVES], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > S2_SPIN_LIMIT) {
            abort = true;
            break;
          }
        }
        if (abort) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      }
      const bool first = k == 0;
      const int g0 = first ? j - (S2_B - 1) : j + 1 + (k - 1) * S2_B;

      // ---- operands
      float x[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = 8 * (hi ? 1 : 0) + i;
        float v = 0.f;
        if (!isD) {
          const int C = g0 + c;
          if (C >= 0) v = ld_nt(AB + (int64_t)C * S2_LD + (S2_B + r - c));
        } else {
          v = r >= c ? ld_nt(AB + (int64_t)(g0 + S2_B + c) * S2_LD + (r - c))
                     : ld_nt(AB + (int64_t)(g0 + S2_B + r) * S2_LD + (c - r));
        }
        x[i] = v;
      }

      // ---- (1) bulge block <- bulge block * H_prev (rows dot v_prev)
      if (!first) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) s += x[i] * vpc[i];
        s += __shfl_xor(s, 16, 64);
        if (!isD) {
          const float f = taup * s;
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] -= f * vpc[i];
        }
      }

      // ---- (2) reflector of the block's first column (task 0: column j)
      const int hgrp = first ? 1 : 0;
      const float hx = first ? x[7] : x[0];
      const float alpha = rdlane(hx, hgrp * 16);
      const float sq = row_sum16((grp == hgrp && r >= 1) ? hx * hx : 0.f);
      const float xn2 = rdlane(sq, hgrp * 16);
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
      const float vr_own = r == 0 ? 1.f : hx * scale;  // valid in group hgrp
      // the new reflector at this lane's 8 columns and at its row
      float v2c[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float lo = rdlane(vr_own, hgrp * 16 + i), up = rdlane(vr_own, hgrp * 16 + 8 + i);
        v2c[i] = hi ? up : lo;
      }
      const float v2r = __shfl(vr_own, hgrp * 16 + r, 64);
      if (grp == hgrp) {
        const float hn = r == 0 ? beta : 0.f;
        if (first) x[7] = hn;
        else x[0] = hn;
      }

      // ---- (3) H v-left-apply to the bulge block's other columns
      if (!first) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float wsum = row_sum16(v2r * x[i]);
          if (!isD && !(grp == 0 && i == 0)) x[i] -= tau * v2r * wsum;
        }
      }

      // ---- (4) diagonal block <- H D H
      float y = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) y += x[i] * v2c[i];
      y += __shfl_xor(y, 16, 64);  // D rows: grp 2 <-> 3
      const float gpart = row_sum16(grp == 2 ? v2r * y : 0.f);
      const float gamma = rdlane(gpart, 32);
      const float z = tau * y - 0.5f * tau * tau * gamma * v2r;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float lo = rdlane(z, 32 + i), up = rdlane(z, 40 + i);
        const float zc = hi ? up : lo;
        if (isD) x[i] -= v2r * zc + z * v2c[i];
      }

      // ---- (5) write back
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = 8 * (hi ? 1 : 0) + i;
        if (!isD) {
          if (!first || (grp == 1 && i == 7))
            AB[(int64_t)(g0 + c) * S2_LD + (S2_B + r - c)] = x[i];
        } else if (r >= c) {
          AB[(int64_t)(g0 + S2_B + c) * S2_LD + (r - c)] = x[i];
        }
      }
      if (grp == hgrp) V2[((int64_t)j * kmax + k) * S2_B + r] = vr_own;
      if (l == 0) tau2s[(int64_t)j * kmax + k] = tau;
#pragma unroll
      for (int i = 0; i < 8; ++i) vpc[i] = v2c[i];
      taup = tau;

      // ---- publish (j, k) done
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (l == 0)
        __hip_atomic_store(&prog[w], j * 65536 + (k + 1 == nk ? 0xFFFF : k + 1),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  if (abort && l == 0) atomicOr(err, 1);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  for (int c = threadIdx.x; c < n; c += S2_T) {
    dout[(int64_t)b * n + c] = ld_nt(AB + (int64_t)c * S2_LD);
    if (c < n - 1) eout[(int64_t)b * (n - 1) + c] = ld_nt(AB + (int64_t)c * S2_LD + 1);
  }
}

}  // namespace

int sb2st_kmax(int n) { return n >= 3 ? 1 + (n - 2) / S2_B : 1; }

void sb2st(float* AB, int64_t sAB, int n, int batch, float* V2, float* tau2, int64_t sV2,
           int kmax, float* d, float* e, int* err, hipStream_t stream) {
  if (batch <= 0 || n <= 0) return;
  hipLaunchKernelGGL(sb2st_kernel, dim3(batch), dim3(S2_T), 0, stream, AB, sAB, n, V2, tau2,
                     sV2, kmax, d, e, err);
}

}  // namespace kfac
