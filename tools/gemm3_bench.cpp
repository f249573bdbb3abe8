// Standalone timing of the grouped bf16x3 GEMM kernel (no torch): the
// ResNet-50 T1 shape set (3 x 512x4608x4608 dominate).  Build variants with
// -DGEMM3_DIAG=N to price phases (see csrc/gemm3.hip).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../csrc/gemm3.hip"

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  struct L { int g, a, cnt; };
  std::vector<L> layers = {{512, 4608, 3}, {256, 2304, 6}, {1000, 2049, 1}, {2048, 1024, 1},
                           {512, 2048, 2}, {2048, 512, 3}, {1024, 256, 6}, {256, 1024, 5},
                           {128, 1152, 4}, {64, 576, 3}, {512, 128, 4}, {128, 512, 3}};
  const bool big_only = argc > 1;
  std::vector<kfac::GemmDesc> descs;
  double flops = 0;
  int tiles = 0;
  for (auto& l : layers) {
    for (int c = 0; c < l.cnt; ++c) {
      if (big_only && l.a != 4608) continue;
      float *A, *B, *C;
      CK(hipMalloc(&A, sizeof(float) * l.g * l.a));
      CK(hipMalloc(&B, sizeof(float) * l.a * l.a));
      CK(hipMalloc(&C, sizeof(float) * l.g * l.a));
      CK(hipMemset(A, 0, sizeof(float) * l.g * l.a));
      CK(hipMemset(B, 0, sizeof(float) * l.a * l.a));
      kfac::GemmDesc d{};
      d.A = A; d.B = B; d.C = C;
      d.lda = l.a; d.ldb = l.a; d.ldc = l.a;
      d.M = l.g; d.N = l.a; d.K = l.a; d.Kmain = l.a;
      d.tiles_n = (l.a + 127) / 128;
      d.tile_start = tiles;
      d.vec = 3;
      tiles += ((l.g + 127) / 128) * d.tiles_n;
      descs.push_back(d);
      flops += 2.0 * l.g * l.a * l.a;
    }
  }
  kfac::GemmDesc* dt;
  CK(hipMalloc(&dt, sizeof(kfac::GemmDesc) * descs.size()));
  CK(hipMemcpy(dt, descs.data(), sizeof(kfac::GemmDesc) * descs.size(), hipMemcpyHostToDevice));
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  for (int w = 0; w < 3; ++w) kfac::gemm3_grouped(dt, (int)descs.size(), tiles, true, false, 0);
  CK(hipEventRecord(s));
  const int iters = 20;
  for (int i = 0; i < iters; ++i) kfac::gemm3_grouped(dt, (int)descs.size(), tiles, true, false, 0);
  CK(hipEventRecord(e));
  CK(hipEventSynchronize(e));
  float ms;
  CK(hipEventElapsedTime(&ms, s, e));
  ms /= iters;
  printf("{\"diag\": %d, \"big_only\": %d, \"tiles\": %d, \"ms\": %.4f, \"tflops\": %.1f}\n",
         GEMM3_DIAG, big_only ? 1 : 0, tiles, ms, flops / ms / 1e9);
  return 0;
}
