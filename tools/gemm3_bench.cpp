// Standalone timing of the grouped bf16x3 GEMM kernel (no torch).
//   gemm3_bench [resnet|neox|big] [akc bkc]
// resnet: the ResNet-50 T1 shape set (3 x 512x4608x4608 dominate);
// neox:   the GPT-NeoX-125M T1 set (12 x {2304x769, 768x769, 3072x769,
//         768x3073} with a bias column, K = a);
// big:    3 x 512x4608x4608 only.
// Operands are filled with random values (MFMA power and clocks depend on
// the data).  Build variants with -DGEMM3_DIAG=N to price phases (see
// csrc/gemm3.hip).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include "../csrc/gemm3.hip"

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); return 1; } } while (0)

__global__ void fill_kernel(float* p, size_t n, unsigned seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = (float)(h & 0xFFFF) / 32768.f - 1.f;
  }
}

int main(int argc, char** argv) {
  struct L { int g, a, cnt, bias; };
  const char* set = argc > 1 ? argv[1] : "resnet";
  const bool akc = argc > 2 ? atoi(argv[2]) != 0 : true;
  const bool bkc = argc > 3 ? atoi(argv[3]) != 0 : false;
  std::vector<L> layers;
  if (!strcmp(set, "neox")) {
    layers = {{2304, 769, 12, 1}, {768, 769, 12, 1}, {3072, 769, 12, 1}, {768, 3073, 12, 1}};
  } else if (!strcmp(set, "big")) {
    layers = {{512, 4608, 3, 0}};
  } else {
    layers = {{512, 4608, 3, 0}, {256, 2304, 6, 0}, {1000, 2049, 1, 1}, {2048, 1024, 1, 0},
              {512, 2048, 2, 0}, {2048, 512, 3, 0}, {1024, 256, 6, 0}, {256, 1024, 5, 0},
              {128, 1152, 4, 0}, {64, 576, 3, 0}, {512, 128, 4, 0}, {128, 512, 3, 0}};
  }
  std::vector<kfac::GemmDesc> descs;
  double flops = 0;
  int tiles = 0;
  unsigned seed = 1;
  for (auto& l : layers) {
    for (int c = 0; c < l.cnt; ++c) {
      // C[g, a] = A[g, a] B[a, a]; A holds the weight gradient (its last
      // column from the bias vector when l.bias), B a dense basis
      const int kmain = l.a - l.bias;
      float *A, *Ax = nullptr, *B, *C;
      CK(hipMalloc(&A, sizeof(float) * l.g * l.a));
      CK(hipMalloc(&B, sizeof(float) * l.a * l.a));
      CK(hipMalloc(&C, sizeof(float) * l.g * l.a));
      fill_kernel<<<1024, 256>>>(A, (size_t)l.g * l.a, seed++);
      fill_kernel<<<1024, 256>>>(B, (size_t)l.a * l.a, seed++);
      if (l.bias) {
        CK(hipMalloc(&Ax, sizeof(float) * l.g));
        fill_kernel<<<64, 256>>>(Ax, (size_t)l.g, seed++);
      }
      kfac::GemmDesc d{};
      d.A = A; d.A_extra = akc ? Ax : nullptr; d.B = B; d.C = C;
      d.lda = akc ? kmain : l.g; d.ldb = l.a; d.ldc = l.a;
      d.M = l.g; d.N = l.a; d.K = l.a; d.Kmain = akc ? kmain : l.a;
      d.tiles_n = (l.a + 127) / 128;
      d.tile_start = tiles;
      d.vec = ((d.lda % 4) == 0 ? 1 : 0) | ((d.ldb % 4) == 0 ? 2 : 0);
      tiles += ((l.g + 127) / 128) * d.tiles_n;
      descs.push_back(d);
      flops += 2.0 * l.g * l.a * l.a;
    }
  }
  CK(hipDeviceSynchronize());
  kfac::GemmDesc* dt;
  CK(hipMalloc(&dt, sizeof(kfac::GemmDesc) * descs.size()));
  CK(hipMemcpy(dt, descs.data(), sizeof(kfac::GemmDesc) * descs.size(), hipMemcpyHostToDevice));
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  for (int w = 0; w < 3; ++w) kfac::gemm3_grouped(dt, (int)descs.size(), tiles, akc, bkc, 0);
  CK(hipEventRecord(s));
  const int iters = 20;
  for (int i = 0; i < iters; ++i) kfac::gemm3_grouped(dt, (int)descs.size(), tiles, akc, bkc, 0);
  CK(hipEventRecord(e));
  CK(hipEventSynchronize(e));
  float ms;
  CK(hipEventElapsedTime(&ms, s, e));
  ms /= iters;
  printf("{\"diag\": %d, \"set\": \"%s\", \"akc\": %d, \"bkc\": %d, \"tiles\": %d, \"ms\": %.4f, "
         "\"fp32_tflops\": %.1f, \"bf16_mfma_tflops\": %.1f}\n",
         GEMM3_DIAG, set, akc ? 1 : 0, bkc ? 1 : 0, tiles, ms, flops / ms / 1e9,
         3 * flops / ms / 1e9);
  return 0;
}
