// Per-dispatch floor of dependent kernels on one stream (MI355X): how much
// of a Householder chain column (two dependent launches, ~16 us at n = 4608)
// is the dispatch itself.  Times N back-to-back launches with HIP events for
//   empty      <<<1, 64>>>            no memory
//   empty_wide <<<1536, 256>>>        no memory, symv-sized grid
//   touch      <<<18, 256>>>          one load + one store per thread (col-sized)
//   touch_wide <<<1536, 256>>>        the same on a symv-sized grid
//   stream     <<<1536, 256>>>        each thread reads 16 floats of a 96 MB matrix
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/launch_floor tools/launch_floor.cpp
//   /tmp/launch_floor [N]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void empty_kernel(float* p) {
  if (p == nullptr && threadIdx.x == 12345) p[0] = 0.f;  // never taken
}

__global__ void touch_kernel(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5f + 1.f;
}

__global__ void stream_kernel(const float* __restrict__ a, float* out, long n) {
  const long base = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const long j = base + u;
    s += j < n ? a[j] : 0.f;
  }
  if (s == 12345.f) out[0] = s;  // keeps the loads
}

template <typename F>
static float timed(F launch, int n, hipStream_t st) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 50; ++i) launch();
  (void)hipStreamSynchronize(st);
  (void)hipEventRecord(a, st);
  for (int i = 0; i < n; ++i) launch();
  (void)hipEventRecord(b, st);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms * 1e3f / n;  // us per launch
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4000;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const long big = 1536L * 256 * 16;  // 6.3M floats = 25 MB (fits the MALL)
  float *buf, *mat;
  CK(hipMalloc(&buf, 1 << 22));
  CK(hipMalloc(&mat, big * sizeof(float)));
  CK(hipMemset(mat, 0, big * sizeof(float)));
  CK(hipMemset(buf, 0, 1 << 22));
  const float t0 = timed([&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, buf); }, n, st);
  const float t1 = timed([&] { hipLaunchKernelGGL(empty_kernel, dim3(1536), dim3(256), 0, st, buf); }, n, st);
  const float t2 = timed([&] { hipLaunchKernelGGL(touch_kernel, dim3(18), dim3(256), 0, st, buf, 18 * 256); }, n, st);
  const float t3 = timed([&] { hipLaunchKernelGGL(touch_kernel, dim3(1536), dim3(256), 0, st, buf, 1536 * 256); }, n, st);
  const float t4 = timed([&] { hipLaunchKernelGGL(stream_kernel, dim3(1536), dim3(256), 0, st, mat, buf, big); }, n, st);
  CK(hipGetLastError());
  printf("{\"launches\": %d, \"us_per_launch\": {\"empty_1x64\": %.3f, \"empty_1536x256\": %.3f, "
         "\"touch_18x256\": %.3f, \"touch_1536x256\": %.3f, \"stream_25MB_1536x256\": %.3f}}\n",
         n, t0, t1, t2, t3, t4);
  CK(hipFree(buf));
  CK(hipFree(mat));
  return 0;
}
