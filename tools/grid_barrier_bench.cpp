// Cost of a device-wide barrier inside one persistent kernel on MI355X: the
// building block of a Householder chain that runs a whole panel (32 columns,
// two barriers per column) per launch instead of two dependent launches per
// column (~16 us at n = 4608, profiles/launch_floor_r4.json).
//
// Each of G workgroups (256 threads) runs `iters` rounds of:
//   write 1 float per thread to a shared vector (system-coherent store),
//   barrier,
//   read 256 floats written by OTHER workgroups and check them.
// Barrier variants:
//   0  agent-scope release/acquire atomics (the compiler's memory model:
//      L2 writeback on release, invalidate on acquire)
//   1  relaxed agent-scope atomics + explicit vmcnt wait; the shared data go
//      through sc1 (L2-bypassing) loads/stores, so no L2 maintenance
//   2  as 1, two-level: blocks arrive on one of 16 group counters, the last
//      arrival of a group on the top counter (fewer serialised atomics on
//      one address); everyone polls the top counter
// Every spin is bounded: after ~2^24 polls a workgroup sets an error flag and
// returns, so a grid that is not co-resident cannot hang the GPU; the host
// also refuses grids larger than the occupancy calculator's resident count.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/gbar tools/grid_barrier_bench.cpp
//   /tmp/gbar [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int T = 256;
constexpr unsigned SPIN_LIMIT = 1u << 24;

__device__ __forceinline__ void st_coherent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_coherent(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int NGRP = 16;

template <int MODE>
__device__ __forceinline__ bool grid_barrier(unsigned* ctr, unsigned target, int* err) {
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    if (MODE == 2) {
      // ctr[0] top, ctr[1 + g] group counters; target = epoch * G
      const unsigned G = gridDim.x, epoch = target / G;
      const unsigned g = blockIdx.x % NGRP;
      const unsigned gsize = G / NGRP + (g < G % NGRP ? 1u : 0u);
      const unsigned ngrp = G < NGRP ? G : NGRP;
      __builtin_amdgcn_s_waitcnt(0);
      const unsigned old =
          __hip_atomic_fetch_add(ctr + 1 + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old + 1 == epoch * gsize)
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned polls = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch * ngrp) {
        __builtin_amdgcn_s_sleep(1);
        if (++polls > SPIN_LIMIT) { ok = false; break; }
      }
    } else if (MODE == 0) {
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      unsigned polls = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++polls > SPIN_LIMIT) { ok = false; break; }
      }
    } else {
      // every store of this workgroup has completed (stores are sc1:
      // they reached the coherence point) before the arrival is counted
      __builtin_amdgcn_s_waitcnt(0);
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned polls = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++polls > SPIN_LIMIT) { ok = false; break; }
      }
    }
    if (!ok) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __shared__ int s_ok;
  if (threadIdx.x == 0) s_ok = ok;
  __syncthreads();
  return s_ok != 0;
}

template <int MODE>
__global__ void __launch_bounds__(T) bar_kernel(float* vec, unsigned* ctr, int* err, int iters,
                                                int* bad) {
  const int G = gridDim.x;
  const int me = blockIdx.x;
  int wrong = 0;
  for (int it = 0; it < iters; ++it) {
    st_coherent(&vec[(size_t)me * T + threadIdx.x], (float)(it * 7 + me));
    if (!grid_barrier<MODE>(ctr, (unsigned)(it + 1) * (unsigned)G, err)) return;
    const int other = (me + 1 + (it % (G > 1 ? G - 1 : 1))) % G;
    const float v = ld_coherent(&vec[(size_t)other * T + threadIdx.x]);
    wrong += v != (float)(it * 7 + other);
    // second barrier: nobody overwrites vec before everyone has read it
    if (!grid_barrier<MODE>(ctr + 32, (unsigned)(it + 1) * (unsigned)G, err)) return;
  }
  if (wrong) atomicAdd(bad, wrong);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  int per_cu0 = 0, per_cu1 = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu0, bar_kernel<0>, T, 0));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu1, bar_kernel<1>, T, 0));
  const int resident = cus * (per_cu0 < per_cu1 ? per_cu0 : per_cu1);
  float* vec;
  unsigned* ctr;
  int *err, *bad;
  CK(hipMalloc(&vec, sizeof(float) * 2048 * T));
  CK(hipMalloc(&ctr, sizeof(unsigned) * 64));
  CK(hipMalloc(&err, sizeof(int)));
  CK(hipMalloc(&bad, sizeof(int)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  printf("{\"cus\": %d, \"resident_blocks\": %d, \"iters\": %d}\n", cus, resident, iters);
  const int grids[] = {1, 8, 32, 64, 128, 256, 512, 1024};
  for (int mode = 0; mode < 3; ++mode) {
    for (int G : grids) {
      if (G > resident || G > 2048) continue;
      CK(hipMemset(ctr, 0, sizeof(unsigned) * 64));
      CK(hipMemset(err, 0, sizeof(int)));
      CK(hipMemset(bad, 0, sizeof(int)));
      CK(hipEventRecord(a, 0));
      if (mode == 0)
        hipLaunchKernelGGL(bar_kernel<0>, dim3(G), dim3(T), 0, 0, vec, ctr, err, iters, bad);
      else if (mode == 1)
        hipLaunchKernelGGL(bar_kernel<1>, dim3(G), dim3(T), 0, 0, vec, ctr, err, iters, bad);
      else
        hipLaunchKernelGGL(bar_kernel<2>, dim3(G), dim3(T), 0, 0, vec, ctr, err, iters, bad);
      CK(hipGetLastError());
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, a, b));
      int herr = 0, hbad = 0;
      CK(hipMemcpy(&herr, err, sizeof(int), hipMemcpyDeviceToHost));
      CK(hipMemcpy(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost));
      printf("{\"mode\": %d, \"grid\": %d, \"us_per_barrier\": %.3f, \"timeout\": %d, "
             "\"wrong\": %d}\n", mode, G, ms * 1e3f / (2.0f * iters), herr, hbad);
      fflush(stdout);
      if (herr) return 2;
    }
  }
  return 0;
}
