// Standalone check + timing of the pre-split grouped GEMM (csrc/gemm3s.hip).
//   gemm3s_bench [neox|resnet|big] [a_mc b_mc out_split [a|g]]
// The last argument picks the inner dimension: K = a (the T1 / T4 tables,
// 2 g a^2 flops per layer) or K = g (T2 / T3, 2 g^2 a).
// Builds random fp32 operands, splits them into images with split_pad_multi,
// runs the grouped GEMM, checks layer 0 against a naive fp64-accumulated
// GEMM and reports the time of the GEMM launch alone.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include "../csrc/gemm3s.hip"

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); return 1; } } while (0)

__global__ void fill_kernel(float* p, size_t n, unsigned seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = (float)(h & 0xFFFF) / 32768.f - 1.f;
  }
}

__global__ void ones_kernel(float* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = 1.f;
}

// C[m][n] = sum_k A(m,k) B(k,n); A(m,k) = amc ? XA[k][m] : XA[m][k]
__global__ void ref_kernel(const float* XA, const float* XB, double* C, int M, int N, int K,
                           int amc, int bmc) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int m = blockIdx.y;
  if (n >= N) return;
  double s = 0.0;
  for (int k = 0; k < K; ++k) {
    const double a = amc ? XA[(size_t)k * M + m] : XA[(size_t)m * K + k];
    const double b = bmc ? XB[(size_t)k * N + n] : XB[(size_t)n * K + k];
    s += a * b;
  }
  C[(size_t)m * N + n] = s;
}

static int64_t r128(int64_t x) { return (x + 255) / 256 * 256; }  // image alignment

int main(int argc, char** argv) {
  struct L { int g, a, cnt; };
  const char* set = argc > 1 ? argv[1] : "neox";
  const bool amc = argc > 2 ? atoi(argv[2]) != 0 : false;
  const bool bmc = argc > 3 ? atoi(argv[3]) != 0 : true;
  const bool osplit = argc > 4 ? atoi(argv[4]) != 0 : false;
  const bool kg = argc > 5 && argv[5][0] == 'g';
  std::vector<L> layers;
  if (!strcmp(set, "neox")) {
    layers = {{2304, 769, 12}, {768, 769, 12}, {3072, 769, 12}, {768, 3073, 12}};
  } else if (!strcmp(set, "big")) {
    layers = {{512, 4608, 3}};
  } else {
    layers = {{512, 4608, 3}, {256, 2304, 6}, {1000, 2049, 1}, {2048, 1024, 1},
              {512, 2048, 2}, {2048, 512, 3}, {1024, 256, 6}, {256, 1024, 5},
              {128, 1152, 4}, {64, 576, 3}, {512, 128, 4}, {128, 512, 3}};
  }
  std::vector<kfac::Gemm3sDesc> descs;
  std::vector<kfac::SplitDesc> sdescs;
  double flops = 0;
  int tiles = 0;
  int64_t sblocks = 0;
  unsigned seed = 1;
  float *XA0 = nullptr, *XB0 = nullptr;
  void* C0 = nullptr;
  int M0 = 0, N0 = 0, K0 = 0;
  int64_t c0_plane = 0, c0_ld = 0;
  for (auto& l : layers) {
    for (int c = 0; c < l.cnt; ++c) {
      const int M = l.g, N = l.a, K = kg ? l.g : l.a;
      const int ar = amc ? K : M, ac = amc ? M : K;   // XA shape
      const int br = bmc ? K : N, bc = bmc ? N : K;   // XB shape
      float *XA, *XB;
      CK(hipMalloc(&XA, sizeof(float) * ar * ac));
      CK(hipMalloc(&XB, sizeof(float) * br * bc));
      fill_kernel<<<1024, 256>>>(XA, (size_t)ar * ac, seed++);
      fill_kernel<<<1024, 256>>>(XB, (size_t)br * bc, seed++);
      uint16_t *IA, *IB;
      const int64_t pa = r128(ar) * r128(ac), pb = r128(br) * r128(bc);
      CK(hipMalloc(&IA, 2 * sizeof(uint16_t) * pa));
      CK(hipMalloc(&IB, 2 * sizeof(uint16_t) * pb));
      CK(hipMemset(IA, 0, 2 * sizeof(uint16_t) * pa));
      CK(hipMemset(IB, 0, 2 * sizeof(uint16_t) * pb));
      for (int o = 0; o < 2; ++o) {
        kfac::SplitDesc s{};
        s.src = o ? XB : XA;
        s.dst = o ? IB : IA;
        s.rows = o ? br : ar;
        s.cols = o ? bc : ac;
        s.lds = s.cols;
        s.ldd = r128(s.cols);
        s.plane = o ? pb : pa;
        s.vec = (s.cols % 4) == 0;
        s.block_start = sblocks;
        sblocks += kfac::split_blocks_for(s.rows, s.cols);
        sdescs.push_back(s);
      }
      void* C;
      const int64_t cld = osplit ? r128(N) : N;
      const int64_t cpl = r128(M) * r128(N);
      CK(hipMalloc(&C, osplit ? 2 * sizeof(uint16_t) * cpl : sizeof(float) * M * N));
      kfac::Gemm3sDesc d{};
      d.A = IA; d.B = IB; d.C = C;
      d.a_plane = pa; d.b_plane = pb; d.c_plane = osplit ? cpl : 0;
      d.lda = r128(ac); d.ldb = r128(bc); d.ldc = cld;
      d.M = M; d.N = N; d.K = K;
      if (getenv("G3S_SCALE") != nullptr) {
        // the T2 epilogue's eigenvalue scaling, by a matrix of ones (the
        // check below stays exact)
        float* S;
        CK(hipMalloc(&S, sizeof(float) * M * N));
        ones_kernel<<<1024, 256>>>(S, (size_t)M * N);
        d.S = S;
        d.lds = N;
      }
      d.tiles_n = (N + kfac::TBN - 1) / kfac::TBN;
      d.tile_start = tiles;
      tiles += ((M + kfac::TBM - 1) / kfac::TBM) * d.tiles_n;
      descs.push_back(d);
      flops += 2.0 * M * N * K;
      if (!XA0) { XA0 = XA; XB0 = XB; C0 = C; M0 = M; N0 = N; K0 = K; c0_plane = cpl; c0_ld = cld; }
    }
  }
  kfac::SplitDesc* sd;
  CK(hipMalloc(&sd, sizeof(kfac::SplitDesc) * sdescs.size()));
  CK(hipMemcpy(sd, sdescs.data(), sizeof(kfac::SplitDesc) * sdescs.size(), hipMemcpyHostToDevice));
  kfac::split_pad_multi(sd, (int)sdescs.size(), sblocks, 0);
  kfac::Gemm3sDesc* dt;
  CK(hipMalloc(&dt, sizeof(kfac::Gemm3sDesc) * descs.size()));
  CK(hipMemcpy(dt, descs.data(), sizeof(kfac::Gemm3sDesc) * descs.size(), hipMemcpyHostToDevice));
  kfac::gemm3s_grouped(dt, (int)descs.size(), tiles, amc, bmc, osplit, 0);
  CK(hipDeviceSynchronize());
  // check layer 0
  double* R;
  CK(hipMalloc(&R, sizeof(double) * M0 * N0));
  ref_kernel<<<dim3((N0 + 255) / 256, M0), 256>>>(XA0, XB0, R, M0, N0, K0, amc, bmc);
  CK(hipDeviceSynchronize());
  std::vector<double> hr((size_t)M0 * N0);
  CK(hipMemcpy(hr.data(), R, sizeof(double) * hr.size(), hipMemcpyDeviceToHost));
  std::vector<float> hc((size_t)M0 * N0);
  if (osplit) {
    std::vector<uint16_t> img(2 * c0_plane);
    CK(hipMemcpy(img.data(), C0, sizeof(uint16_t) * img.size(), hipMemcpyDeviceToHost));
    auto bf = [](uint16_t u) { uint32_t x = (uint32_t)u << 16; float f; memcpy(&f, &x, 4); return f; };
    for (int m = 0; m < M0; ++m)
      for (int n = 0; n < N0; ++n)
        hc[(size_t)m * N0 + n] = bf(img[m * c0_ld + n]) + bf(img[c0_plane + m * c0_ld + n]);
  } else {
    CK(hipMemcpy(hc.data(), C0, sizeof(float) * hc.size(), hipMemcpyDeviceToHost));
  }
  double maxref = 0, maxerr = 0;
  for (size_t i = 0; i < hr.size(); ++i) {
    maxref = fmax(maxref, fabs(hr[i]));
    maxerr = fmax(maxerr, fabs(hr[i] - (double)hc[i]));
  }
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  for (int w = 0; w < 3; ++w) kfac::gemm3s_grouped(dt, (int)descs.size(), tiles, amc, bmc, osplit, 0);
  CK(hipEventRecord(s));
  const int iters = 20;
  for (int i = 0; i < iters; ++i) kfac::gemm3s_grouped(dt, (int)descs.size(), tiles, amc, bmc, osplit, 0);
  CK(hipEventRecord(e));
  CK(hipEventSynchronize(e));
  float ms;
  CK(hipEventElapsedTime(&ms, s, e));
  ms /= iters;
  // the per-step split of one operand set (what the W split costs)
  CK(hipEventRecord(s));
  for (int i = 0; i < iters; ++i) kfac::split_pad_multi(sd, (int)sdescs.size(), sblocks, 0);
  CK(hipEventRecord(e));
  CK(hipEventSynchronize(e));
  float sms;
  CK(hipEventElapsedTime(&sms, s, e));
  sms /= iters;
  printf("{\"set\": \"%s\", \"k\": \"%s\", \"a_mc\": %d, \"b_mc\": %d, \"out_split\": %d, \"tiles\": %d, \"ms\": %.4f, "
         "\"fp32_tflops\": %.1f, \"bf16_mfma_tflops\": %.1f, \"rel_err\": %.3e, \"split_all_ms\": %.4f}\n",
         set, kg ? "g" : "a", amc ? 1 : 0, bmc ? 1 : 0, osplit ? 1 : 0, tiles, ms, flops / ms / 1e9,
         3 * flops / ms / 1e9, maxerr / maxref, sms);
  return (maxerr / maxref < 5e-5) ? 0 : 2;
}
