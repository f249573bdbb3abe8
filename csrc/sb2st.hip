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
// task (j, k) only has to follow task (j, k-1) and task (j-1, k+2) (the
// float64 oracle, ops/twostage.py sb2st_reference(order='pipeline'), replays
// any schedule with that rule and matches the sequential order bit for bit).
//
// Work layout: one 768-thread workgroup per matrix (12 waves, 150 VGPRs: no
// spills); each wave runs FOUR
// sweeps at once, one per 16-lane DPP row ("group"), lane r of a group owning
// row r of the task's bulge block and of its diagonal block (16 + 16 values).
// The four groups advance in lockstep, group g executing task k = t - 4g at
// step t: a lag of four tasks (one more than the dependency rule needs), so
// the operands of step t+1 were written two steps earlier and are loaded
// while step t computes.  Row reductions are DPP row sums, column sums and
// broadcasts go through the wave's LDS slice.  Wave w runs sweeps
// 48 rho + 4 w + g in round rho; the first group of a wave follows the last
// group of the previous wave through per-wave progress words in LDS
// (workgroup-scope release / acquire; band loads bypass L1).  The band lives
// in L2-resident global memory, column-major with 32 distances per column
// (AB[c][d] = B[c+d][c]); padding columns past n are zero.  Reflectors
// (v[0] = 1 stored, tau) go to V2[j][k][16] / tau2[j][k] for the
// back-transform (csrc/bt2.hip).
#include "common.h"

namespace kfac {

namespace {

constexpr int S2_B = 16;
constexpr int S2_LD = 2 * S2_B;   // band storage: distances 0..31 per column
constexpr int S2_WAVES = 12;
constexpr int S2_T = 64 * S2_WAVES;
constexpr int S2_LAG = 4;         // tasks between consecutive sweeps
constexpr int S2_SPIN_LIMIT = 1 << 24;  // ~1 s: a correct run waits microseconds
constexpr int S2_RS = 1 << 20;    // progress word: round * S2_RS + steps done
constexpr int S2_TLD = 20;        // LDS transpose row stride (16-B aligned rows)
constexpr int S2_GST = S2_B * S2_TLD + 16;  // LDS words per group slice

__device__ __forceinline__ int ntasks(int j, int n) { return 1 + (n - 2 - j) / S2_B; }

// sum over the 16 lanes of each DPP row, left in every lane of the row
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_mov<0xb1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_mov<0x4e>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v;
}

__device__ __forceinline__ float ld_nt(const float* p) { return __builtin_nontemporal_load(p); }

struct Task {
  int j, k, g0;
  bool on;
};

__device__ __forceinline__ Task task_of(int rho, int w, int g, int t, int n) {
  Task s;
  s.j = 4 * S2_WAVES * rho + 4 * w + g;
  s.k = t - S2_LAG * g;
  s.on = s.j < n - 2 && s.k >= 0 && s.k < ntasks(s.j, n);
  s.g0 = s.k == 0 ? s.j - (S2_B - 1) : s.j + 1 + (s.k - 1) * S2_B;
  return s;
}

// bulge-block row r (task 0: only its last column, column j) and diagonal
// block row r (both triangles from the symmetric band storage)
__device__ __forceinline__ void load_task(const float* AB, const Task& s, int r,
                                          float (&bk)[S2_B], float (&dd)[S2_B]) {
#pragma unroll
  for (int c = 0; c < S2_B; ++c) {
    bk[c] = 0.f;
    dd[c] = 0.f;
  }
  if (!s.on) return;
  if (s.k == 0) {
    bk[S2_B - 1] = ld_nt(AB + (int64_t)(s.g0 + S2_B - 1) * S2_LD + (r + 1));
  } else {
#pragma unroll
    for (int c = 0; c < S2_B; ++c) bk[c] = ld_nt(AB + (int64_t)(s.g0 + c) * S2_LD + (S2_B + r - c));
  }
  // lower triangle only (coalesced: lanes r of column c are consecutive
  // words); the upper triangle comes from the transpose in fill_upper
#pragma unroll
  for (int c = 0; c < S2_B; ++c)
    if (r >= c) dd[c] = ld_nt(AB + (int64_t)(s.g0 + S2_B + c) * S2_LD + (r - c));
}

// dd[c] for c > r from the other lanes' lower rows (LDS transpose): the
// upper-triangle band words of a row are 31 floats apart, one cache line per
// lane -- loading them directly made the bulge chase VMEM-bound
__device__ __forceinline__ void fill_upper(float* tbg, int r, float (&dd)[S2_B]) {
#pragma unroll
  for (int c = 0; c < S2_B; ++c)
    if (c <= r) tbg[r * S2_TLD + c] = dd[c];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int c = 0; c < S2_B; ++c)
    if (c > r) dd[c] = tbg[c * S2_TLD + r];
  __builtin_amdgcn_wave_barrier();
}

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
  // per-group transpose slices; group stride 336 words = 16 banks apart, so
  // the four groups of a wave never collide
  __shared__ __attribute__((aligned(16))) float tb[S2_WAVES][4 * S2_GST];
  __shared__ __attribute__((aligned(16))) float bc[S2_WAVES][4][S2_B];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int r = l & 15, g = l >> 4;
  float* tbg = &tb[w][g * S2_GST];
  float* bcg = &bc[w][g][0];
  if (l == 0) prog[w] = -1;
  __syncthreads();
  bool abort = false;
  const int nsweep = n - 2;
  const int rounds = (nsweep + 4 * S2_WAVES - 1) / (4 * S2_WAVES);
  const int pw = (w + S2_WAVES - 1) % S2_WAVES;

  // waits until the previous sweep (last group of the previous wave) has
  // finished task q (its round prho); q >= its task count means "finished"
  auto wait_pred = [&](int prho, int q) {
    const int target = prho * S2_RS + q + 1 + S2_LAG * 3;
    int spins = 0;
    while (__hip_atomic_load(&prog[pw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <
           target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > S2_SPIN_LIMIT) {
        abort = true;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };

  for (int rho = 0; rho < rounds && !abort; ++rho) {
    const int j0 = 4 * S2_WAVES * rho + 4 * w;  // this wave's group-0 sweep
    if (j0 >= nsweep) break;
    int steps = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int jq = j0 + q;
      if (jq < nsweep) steps = max(steps, S2_LAG * q + ntasks(jq, n));
    }
    const int prho = w == 0 ? rho - 1 : rho;
    const bool has_pred = j0 > 0;
    const int nkp = has_pred ? ntasks(j0 - 1, n) : 0;
    float bk[S2_B], dd[S2_B], nbk[S2_B], ndd[S2_B], vp[S2_B];
    float taup = 0.f;
#pragma unroll
    for (int c = 0; c < S2_B; ++c) vp[c] = 0.f;
    // operands of step 0 (group 0's task 0 needs the previous sweep's task 2)
    if (has_pred) wait_pred(prho, min(2, nkp - 1));
    if (abort) break;
    load_task(AB, task_of(rho, w, g, 0, n), r, bk, dd);
    for (int t = 0; t < steps; ++t) {
      const Task s = task_of(rho, w, g, t, n);
      fill_upper(tbg, r, dd);
      // ---- prefetch step t+1 (written at step t-1 or earlier: complete)
      if (has_pred && t + 1 < steps) {
        const int k1 = t + 1;  // group 0's next task
        if (k1 < ntasks(j0, n)) wait_pred(prho, min(k1 + 2, nkp - 1));
        if (abort) break;
      }
      load_task(AB, task_of(rho, w, g, t + 1, n), r, nbk, ndd);
      const bool first = s.k == 0;

      // ---- (1) bulge block <- bulge block * H_prev (row r dot v_prev)
      if (!first) {
        float sdot = 0.f;
#pragma unroll
        for (int c = 0; c < S2_B; ++c) sdot += bk[c] * vp[c];
        const float f = taup * sdot;
#pragma unroll
        for (int c = 0; c < S2_B; ++c) bk[c] -= f * vp[c];
      }
      // ---- (2) reflector of the block's first column (task 0: column j)
      const float hx = first ? bk[S2_B - 1] : bk[0];
      const float alpha = row_sum16(r == 0 ? hx : 0.f);
      const float xn2 = row_sum16(r >= 1 ? hx * hx : 0.f);
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
      const float v2r = r == 0 ? 1.f : hx * scale;
      const float hn = r == 0 ? beta : 0.f;
      if (first) bk[S2_B - 1] = hn;
      else bk[0] = hn;
      // broadcast v2 to the group (vp is dead from here on: reuse it)
      bcg[r] = v2r;
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int q = 0; q < S2_B / 4; ++q) {
        const float4 v4 = reinterpret_cast<const float4*>(bcg)[q];
        vp[4 * q] = v4.x;
        vp[4 * q + 1] = v4.y;
        vp[4 * q + 2] = v4.z;
        vp[4 * q + 3] = v4.w;
      }
      __builtin_amdgcn_wave_barrier();
      // ---- (3) H left-applied to the bulge block's other columns
      if (!first) {
#pragma unroll
        for (int q = 0; q < S2_B / 4; ++q)
          reinterpret_cast<float4*>(tbg + r * S2_TLD)[q] =
              make_float4(v2r * bk[4 * q], v2r * bk[4 * q + 1], v2r * bk[4 * q + 2],
                          v2r * bk[4 * q + 3]);
        __builtin_amdgcn_wave_barrier();
        float wcol = 0.f;  // column r sum
#pragma unroll
        for (int q = 0; q < S2_B; ++q) wcol += tbg[q * S2_TLD + r];
        __builtin_amdgcn_wave_barrier();
        tbg[r] = wcol;  // row 0 of the slice is free again (every lane read it)
        __builtin_amdgcn_wave_barrier();
        const float f = tau * v2r;
#pragma unroll
        for (int q = 0; q < S2_B / 4; ++q) {
          const float4 w4 = reinterpret_cast<const float4*>(tbg)[q];
          if (q > 0) bk[4 * q] -= f * w4.x;  // column 0 holds the reflector
          bk[4 * q + 1] -= f * w4.y;
          bk[4 * q + 2] -= f * w4.z;
          bk[4 * q + 3] -= f * w4.w;
        }
        __builtin_amdgcn_wave_barrier();
      }
      // ---- (4) diagonal block <- H D H
      float y = 0.f;
#pragma unroll
      for (int c = 0; c < S2_B; ++c) y += dd[c] * vp[c];
      const float gamma = row_sum16(v2r * y);
      const float z = tau * y - 0.5f * tau * tau * gamma * v2r;
      bcg[r] = z;
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int q = 0; q < S2_B / 4; ++q) {
        const float4 z4 = reinterpret_cast<const float4*>(bcg)[q];
        dd[4 * q] -= v2r * z4.x + z * vp[4 * q];
        dd[4 * q + 1] -= v2r * z4.y + z * vp[4 * q + 1];
        dd[4 * q + 2] -= v2r * z4.z + z * vp[4 * q + 2];
        dd[4 * q + 3] -= v2r * z4.w + z * vp[4 * q + 3];
      }
      __builtin_amdgcn_wave_barrier();
      // ---- (5) write back
      if (s.on) {
        if (first) {
          AB[(int64_t)(s.g0 + S2_B - 1) * S2_LD + (r + 1)] = bk[S2_B - 1];
        } else {
#pragma unroll
          for (int c = 0; c < S2_B; ++c)
            AB[(int64_t)(s.g0 + c) * S2_LD + (S2_B + r - c)] = bk[c];
        }
#pragma unroll
        for (int c = 0; c < S2_B; ++c)
          if (c <= r) AB[(int64_t)(s.g0 + S2_B + c) * S2_LD + (r - c)] = dd[c];
        V2[((int64_t)s.j * kmax + s.k) * S2_B + r] = v2r;
        if (r == 0) tau2s[(int64_t)s.j * kmax + s.k] = tau;
      }
      taup = tau;
      // ---- publish step t (its stores, and the prefetch, complete)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (l == 0)
        __hip_atomic_store(&prog[w], rho * S2_RS + t + 1, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
      for (int c = 0; c < S2_B; ++c) {
        bk[c] = nbk[c];
        dd[c] = ndd[c];
      }
    }
    if (l == 0)
      __hip_atomic_store(&prog[w], rho * S2_RS + (S2_RS - 1), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  if (abort && l == 0) atomicOr(err + b, 1);  // this matrix only
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
