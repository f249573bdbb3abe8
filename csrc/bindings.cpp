#include <cstdlib>
#include <string>
// Python bindings for the MI355X K-FAC kernels (module
// distributed_kfac_pytorch_amd._C).  This is the only translation unit that
// includes torch; it validates tensors, picks the current HIP stream and
// calls the raw launchers in the *.hip files.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <tuple>
#include <vector>

#include "common.h"
#include "descs.h"

namespace kfac {
// pack.hip
void triu_pack(int dtype, const void* src, int64_t ld, int64_t n, void* dst,
               hipStream_t s);
void triu_unpack(int dtype, const void* packed, int64_t n, void* dst,
                 int64_t ld, float scale, hipStream_t s);
void scale_copy(int dtype, const void* src, void* dst, int64_t n, float scale,
                hipStream_t s);
// syrk.hip
int64_t syrk_workspace_splits(int64_t N, int64_t D);
int64_t syrk_workspace_floats(int64_t D, int64_t splits);
void syrk(int in_dtype, const void* x, int64_t N, int64_t K, int64_t ldx,
          bool bias, float* C, int64_t D, int64_t ldc, float alpha,
          float beta, int splits, hipStream_t s, const ConvGeom* geom,
          float* ws, const float* ascale, bool fp32_exact);
void syrk_split_planes(const float* x, int64_t B, int H, int W, int C, int64_t sB, int64_t sH,
                       int64_t sW, uint16_t* planes, hipStream_t s);
// im2col.hip
void im2col_nhwc(int dtype, const void* x, int64_t B, int64_t H, int64_t W,
                 int64_t C, int64_t sB, int64_t sH, int64_t sW, int kh, int kw,
                 int sh, int sw, int ph, int pw, int64_t OH, int64_t OW,
                 void* out, int64_t ldo, int out_dtype, hipStream_t s);
void im2col_nchw(int dtype, const void* x, int64_t B, int64_t C, int64_t H,
                 int64_t W, int64_t sB, int64_t sC, int64_t sH, int64_t sW,
                 int kh, int kw, int sh, int sw, int ph, int pw, int64_t OH,
                 int64_t OW, void* out, int64_t ldo, int out_dtype,
                 hipStream_t s);
// precond.hip
void eigen_scale(float* v, int64_t rows, int64_t cols, int64_t ldv,
                 const float* dgda, const float* dg, const float* da,
                 float damping, hipStream_t s);
void kl_dot_accumulate(const float* p, int64_t rows, int64_t cols, int64_t ldp,
                       const void* wgrad, int wdtype, int64_t ldw,
                       const void* bgrad, int bdtype, double* acc,
                       hipStream_t s);
void kl_scale_finalize(const double* acc, float* scale_out, float kl_clip,
                       float lr, hipStream_t s);
void apply_grad(const float* p, int64_t rows, int64_t cols, int64_t ldp,
                void* wgrad, int wdtype, int64_t ldw, void* bgrad, int bdtype,
                const float* scale, hipStream_t s);
void fill_identity_lerp(float* C, int64_t n, int64_t ldc, hipStream_t s);
// eigh_jacobi.hip
int jacobi_max_n();
void jacobi_eigh_batched(const float* A, int64_t n, int64_t batch,
                         int64_t strideA, float* evals, float* evecs,
                         int64_t strideV, int max_sweeps, float tol,
                         hipStream_t s);
// multi.hip
int64_t multi_blocks_for(int64_t rows, int64_t cols);
void kl_dot_multi(const LayerDesc* descs, int nlayers, int64_t total_blocks,
                  double* acc, hipStream_t s);
void kl_finalize_dev(const double* acc, int64_t nparts, const float* params,
                     float* scale, hipStream_t s);
void kl_reduce_partials(const double* acc, int64_t nparts, double* out, hipStream_t s);
void apply_multi(const LayerDesc* descs, int nlayers, int64_t total_blocks,
                 const float* scale, hipStream_t s);
// gemm3.hip
int gemm3_grid(int total_tiles);
void gemm3_single(const GemmDesc& d, bool a_kc, bool b_kc, int splits, int64_t split_stride,
                  hipStream_t s);
void subsample_fwd(const float* x, float* y, int N, int H, int W, int C, int sh, int sw,
                   hipStream_t s);
void sum_splits(const float* part, float* out, int S, int64_t T, hipStream_t s);
void subsample_bwd(const float* g, float* gx, int N, int H, int W, int C, int sh, int sw,
                   hipStream_t s);
void subsample_bwd_acc(const float* g, float* gx, int N, int H, int W, int C, int sh, int sw,
                   hipStream_t s);
void pad_channels4(const float* x, float* y, int64_t pixels, int C, hipStream_t s);
int gemm3_conv_splits(int N, int H, int W, int C, int Cout, int kh, int kw, int stride, int pad);
void maxpool_nhwc_fwd(int dtype, const void* x, void* y, uint8_t* code, int N, int H, int W,
                      int C, int OH, int OW, int k, int s, int p, hipStream_t st);
void maxpool_nhwc_bwd(int dtype, const void* gy, const uint8_t* code, void* gx, int N, int H,
                      int W, int C, int OH, int OW, int k, int s, int p, hipStream_t st);
void col2im_nhwc(int dtype, const void* cols, void* gx, int B, int H, int W, int C, int OH,
                 int OW, int kh, int kw, int sh, int sw, int ph, int pw, hipStream_t s);
int gemm3_wgrad_splits(int pixels, int Cout, int kcols);
void gemm3_conv_wgrad(const float* x, const float* dy, float* dw, int N, int H, int W, int C,
                      int Cout, int kh, int kw, int stride, int pad, int splits, hipStream_t s);
void gemm3_conv(const float* x, const float* w, float* y, int N, int H, int W, int C, int Cout,
                int kh, int kw, int stride, int pad, int splits, bool flipw, hipStream_t s,
                float* bnpart = nullptr);
void gemm3_grouped(const GemmDesc* table, int nlayers, int total_tiles,
                   bool a_kc, bool b_kc, hipStream_t s);
// gemm3s.hip
int gemm3s_align();
int gemm3s_tile_m();
int gemm3s_tile_n();
int gemm3s_grid(int total_tiles);
int64_t split_blocks_for(int64_t rows, int64_t total_cols);
void gemm3s_grouped(const Gemm3sDesc* table, int nlayers, int total_tiles, bool a_mc,
                    bool b_mc, bool out_split, hipStream_t s);
void split_pad_multi(const SplitDesc* table, int n, int64_t total_blocks, hipStream_t s);
// cast.hip
int64_t cast_blocks_for(int64_t n);
void cast_multi(const CastDesc* table, int n, int64_t total_blocks, bool to_bf16, hipStream_t s);
// bnact.hip
void bn_partition(int64_t M, int C, int64_t* rows_per_block, int* nblk);
int bn_max_c();
void bn_forward(int dtype, const void* x, const void* res, const float* weight,
                const float* bias, float* running_mean, float* running_var,
                int64_t* num_batches, float momentum, float eps, int relu, int64_t M,
                int C, float* part, float* stats, void* y, hipStream_t s,
                const float* ext_part = nullptr, int ext_p = 0);
void bn_backward(int dtype, const void* x, const void* dy, const void* y, const float* weight,
                 const float* stats, int relu, int64_t M, int C, float* part, float* coef,
                 float* dweight, float* dbias, void* dx, void* dres, hipStream_t s);
}  // namespace kfac

// solver.cpp
std::vector<at::Tensor> rocsolver_eigh(at::Tensor A, int64_t algo,
                                       int64_t max_sweeps, double tol);
int64_t sytrd_panel();
int64_t sytrd_max_n();
std::vector<at::Tensor> spd_inverse_blocked(at::Tensor F, double damping);
std::vector<at::Tensor> sytrd_reduce(std::vector<at::Tensor> stacks);
std::vector<at::Tensor> sytrd_begin(std::vector<at::Tensor> stacks);
void sytrd_advance(at::Tensor descs, std::vector<int64_t> sizes, int64_t k0, int64_t k1,
                   int64_t waves);

namespace kfac {
// gemm_f32.hip
void gemm_f32_batched(int ta, int tb, int M, int N, int K, float alpha, const float* A,
                      int64_t lda, int64_t sA, const float* B, int64_t ldb, int64_t sB,
                      float beta, float* C, int64_t ldc, int64_t sC, int batch,
                      hipStream_t s, float* ws, int64_t ws_floats);
int64_t gemm_f32_ws_floats(int M, int N, int K, int batch);
void trinv_upper_batched(float* T, int64_t ld, int64_t sT, int n, int batch, float* work,
                         hipStream_t s);
}  // namespace kfac

namespace {
// native fp32 MFMA GEMM (csrc/gemm_f32.hip) with its split-K workspace
// KFAC_GEMM_IMPL=lib: the same GEMM through ATen's batched matmul (hipBLASLt)
// -- an A/B switch for measurements, not a default
bool gemm_use_lib() {
  static const bool lib = [] {
    const char* e = std::getenv("KFAC_GEMM_IMPL");
    return e != nullptr && std::string(e) == "lib";
  }();
  return lib;
}

void gemm_native(int ta, int tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
                 int64_t lda, int64_t sA, const float* B, int64_t ldb, int64_t sB, float beta,
                 float* C, int64_t ldc, int64_t sC, int64_t batch, hipStream_t s,
                 const at::TensorOptions& opt) {
  if (gemm_use_lib()) {
    auto o = opt.dtype(at::kFloat);
    // ATen launches on the current stream: make it the caller's stream
    at::hip::HIPStreamGuardMasqueradingAsCUDA sg(
        at::hip::getStreamFromExternalMasqueradingAsCUDA(s, opt.device().index()));
    // op(A) [batch, M, K], op(B) [batch, K, N], C [batch, M, N] as strided views
    at::Tensor a = ta ? at::from_blob(const_cast<float*>(A), {batch, M, K}, {sA, 1, lda}, o)
                      : at::from_blob(const_cast<float*>(A), {batch, M, K}, {sA, lda, 1}, o);
    at::Tensor b = tb ? at::from_blob(const_cast<float*>(B), {batch, K, N}, {sB, 1, ldb}, o)
                      : at::from_blob(const_cast<float*>(B), {batch, K, N}, {sB, ldb, 1}, o);
    at::Tensor c = at::from_blob(C, {batch, M, N}, {sC, ldc, 1}, o);
    if (beta == 0.f) {
      at::Tensor r = at::bmm(a, b);
      if (alpha != 1.f) r.mul_(alpha);
      c.copy_(r);
    } else {
      c.baddbmm_(a, b, beta, alpha);
    }
    return;
  }
  const int64_t wsf = kfac::gemm_f32_ws_floats((int)M, (int)N, (int)K, (int)batch);
  at::Tensor ws;
  if (wsf > 0) ws = at::empty({wsf}, opt.dtype(at::kFloat));
  kfac::gemm_f32_batched(ta, tb, (int)M, (int)N, (int)K, alpha, A, lda, sA, B, ldb, sB, beta, C,
                         ldc, sC, (int)batch, s, wsf > 0 ? ws.data_ptr<float>() : nullptr, wsf);
}
}  // namespace


namespace {

hipStream_t cur_stream() {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
}

int dtype_tag(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return kfac::kF32;
    case at::kBFloat16: return kfac::kBF16;
    case at::kDouble: return kfac::kF64;
    case at::kHalf: return kfac::kF16;
    default:
      TORCH_CHECK(false, "kfac native: unsupported dtype ", t.scalar_type());
  }
  return -1;
}

void check_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "kfac native: ", name, " must be a GPU tensor");
}

// ---------------------------------------------------------------- pack
void triu_pack(const at::Tensor& src, at::Tensor& dst) {
  check_cuda(src, "src");
  check_cuda(dst, "dst");
  TORCH_CHECK(src.dim() == 2 && src.size(0) == src.size(1), "square src");
  TORCH_CHECK(src.stride(1) == 1, "src rows must be contiguous");
  TORCH_CHECK(dst.is_contiguous() && dst.scalar_type() == src.scalar_type());
  const int64_t n = src.size(0);
  TORCH_CHECK(dst.numel() == n * (n + 1) / 2, "dst size");
  c10::hip::HIPGuardMasqueradingAsCUDA g(src.device());
  kfac::triu_pack(dtype_tag(src), src.data_ptr(), src.stride(0), n,
                  dst.data_ptr(), cur_stream());
}

void triu_unpack(at::Tensor& dst, const at::Tensor& packed, double scale) {
  check_cuda(dst, "dst");
  check_cuda(packed, "packed");
  TORCH_CHECK(dst.dim() == 2 && dst.size(0) == dst.size(1), "square dst");
  TORCH_CHECK(dst.stride(1) == 1, "dst rows must be contiguous");
  TORCH_CHECK(packed.is_contiguous() &&
              packed.scalar_type() == dst.scalar_type());
  const int64_t n = dst.size(0);
  TORCH_CHECK(packed.numel() == n * (n + 1) / 2, "packed size");
  c10::hip::HIPGuardMasqueradingAsCUDA g(dst.device());
  kfac::triu_unpack(dtype_tag(dst), packed.data_ptr(), n, dst.data_ptr(),
                    dst.stride(0), (float)scale, cur_stream());
}

void scale_copy(at::Tensor& dst, const at::Tensor& src, double scale) {
  check_cuda(dst, "dst");
  check_cuda(src, "src");
  TORCH_CHECK(dst.is_contiguous() && src.is_contiguous());
  TORCH_CHECK(dst.numel() == src.numel());
  TORCH_CHECK(dst.scalar_type() == src.scalar_type());
  c10::hip::HIPGuardMasqueradingAsCUDA g(dst.device());
  kfac::scale_copy(dtype_tag(dst), src.data_ptr(), dst.data_ptr(),
                   dst.numel(), (float)scale, cur_stream());
}

// ---------------------------------------------------------------- syrk
// Split-K partial-tile workspace (stream-ordered caching-allocator memory;
// inside a HIP-graph capture it comes from the graph's private pool).
at::Tensor syrk_ws(const at::Tensor& C, int64_t D, int64_t splits) {
  const int64_t n = kfac::syrk_workspace_floats(D, splits);
  if (n == 0) return at::Tensor();
  return at::empty({n}, C.options());
}

// C[D,D] = beta*C + alpha * Xt^T Xt, Xt = [X | 1] when bias.
// C: dense [D, D] (unit column stride), or the packed upper triangle
// [D (D + 1) / 2] (the factor all-reduce wire): returns the ldc to pass to
// kfac::syrk (0 = packed)
int64_t syrk_out_ld(const at::Tensor& C, int64_t D) {
  TORCH_CHECK(C.scalar_type() == at::kFloat, "syrk output must be fp32");
  if (C.dim() == 1) {
    TORCH_CHECK(C.numel() == D * (D + 1) / 2 && C.is_contiguous(),
                "packed syrk output must hold D(D+1)/2 contiguous floats");
    return 0;
  }
  TORCH_CHECK(C.dim() == 2 && C.size(0) == D && C.size(1) == D && C.stride(1) == 1,
              "syrk output must be [D, D] with unit column stride");
  return C.stride(0);
}

// ascale: optional 1-element fp32 device tensor multiplying alpha (read by
// the kernel: no host sync for a device-side AMP loss-scale correction)
const float* syrk_ascale(const c10::optional<at::Tensor>& ascale, const at::Tensor& C) {
  if (!ascale.has_value() || !ascale->defined()) return nullptr;
  TORCH_CHECK(ascale->scalar_type() == at::kFloat && ascale->numel() >= 1 &&
                  ascale->device() == C.device(),
              "alpha_scale must be a float32 tensor on the output's device");
  return ascale->data_ptr<float>();
}

void syrk(const at::Tensor& x, at::Tensor& C, bool bias, double alpha,
          double beta, int64_t splits, const c10::optional<at::Tensor>& ascale,
          bool fp32_exact) {
  check_cuda(x, "x");
  check_cuda(C, "C");
  TORCH_CHECK(x.dim() == 2, "x must be 2D [N, K]");
  TORCH_CHECK(x.stride(1) == 1, "x rows must be contiguous (stride(1)==1)");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 ||
                  x.scalar_type() == at::kFloat,
              "syrk input must be bf16 or fp32");
  const int64_t N = x.size(0), K = x.size(1);
  const int64_t D = K + (bias ? 1 : 0);
  const int64_t ldc = syrk_out_ld(C, D);
  const int64_t ldx = N > 1 ? x.stride(0) : K;
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  int sp = splits > 0 ? (int)splits : (int)kfac::syrk_workspace_splits(N, D);
  at::Tensor ws = syrk_ws(C, D, sp);
  // fp32 input on the bf16x3 path with several column tiles: every element
  // is otherwise split to bf16 hi / lo once per column tile that reads it
  // (VALU-bound: 45-50 TFLOP/s at D = 1024-2048 vs 110-180 for the
  // pre-split patch SYRKs, profiles/r6/syrk_dense_planes/).  Split it once
  // into contiguous planes and run the planes kernel as a 1x1 "convolution"
  // over a 1x1 image per row, when the input has >= 2M elements (below it
  // the extra pass costs more than it saves: 1568 x 512 went 28 -> 30 us).
  // KFAC_SYRK_DENSE_PLANES_MIN_D: smallest D (default 129, two or more
  // tiles: 100352 x 256 went 203 -> 157 us); 0 disables.
  static const int64_t planes_min_d = [] {
    const char* e = std::getenv("KFAC_SYRK_DENSE_PLANES_MIN_D");
    return e != nullptr ? (int64_t)std::atoll(e) : (int64_t)129;
  }();
  const int64_t elems = N * K;
  if (x.scalar_type() == at::kFloat && !fp32_exact && planes_min_d > 0 && D >= planes_min_d &&
      K % 8 == 0 && ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 &&
      N < (1LL << 24) && elems >= (1LL << 21) && elems < (1LL << 29)) {
    at::Tensor planes = at::empty({2 * elems}, x.options().dtype(at::kBFloat16));
    kfac::syrk_split_planes(x.data_ptr<float>(), N, 1, 1, (int)K, ldx, K, K,
                            reinterpret_cast<uint16_t*>(planes.data_ptr()), cur_stream());
    kfac::ConvGeom gp{K, K, K, 1, 1, (int32_t)K, 1, 1, 1, 0, 0, 1, 1, elems, 0};
    kfac::syrk(kfac::kF32, planes.data_ptr(), N, K, /*ldx=*/K, bias, C.data_ptr<float>(), D,
               ldc, (float)alpha, (float)beta, sp, cur_stream(), &gp,
               ws.defined() ? ws.data_ptr<float>() : nullptr, syrk_ascale(ascale, C), false);
    return;
  }
  kfac::syrk(dtype_tag(x), x.data_ptr(), N, K, ldx, bias,
             C.data_ptr<float>(), D, ldc, (float)alpha, (float)beta,
             sp, cur_stream(), nullptr, ws.defined() ? ws.data_ptr<float>() : nullptr,
             syrk_ascale(ascale, C), fp32_exact);
}

// C[D,D] = beta*C + alpha * P^T P with P the (implicit) patch matrix of an
// NHWC conv input x [B, C, H, W] (channels_last strides), columns in natural
// (kh, kw, c) order, plus the bias ones column.  The patches are read from x
// inside the SYRK tile loader (K-HIP-2: no im2col buffer).
void syrk_conv(const at::Tensor& x, at::Tensor& C, int64_t kh, int64_t kw,
               int64_t sh, int64_t sw, int64_t ph, int64_t pw, bool bias,
               double alpha, double beta, int64_t splits,
               const c10::optional<at::Tensor>& ascale, bool fp32_exact) {
  check_cuda(x, "x");
  check_cuda(C, "C");
  TORCH_CHECK(x.dim() == 4, "x must be [B, C, H, W]");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat,
              "syrk_conv input must be bf16 or fp32");
  const int64_t B = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t vec = x.scalar_type() == at::kFloat ? 4 : 8;  // elements per 16 B
  TORCH_CHECK(x.stride(1) == 1, "syrk_conv needs channels_last input (channel stride 1)");
  TORCH_CHECK(Cin % vec == 0 && x.stride(0) % vec == 0 && x.stride(2) % vec == 0 &&
                  x.stride(3) % vec == 0 &&
                  (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0,
              "syrk_conv: channel count and strides must allow 16-byte loads");
  const int64_t OH = (H + 2 * ph - kh) / sh + 1, OW = (W + 2 * pw - kw) / sw + 1;
  TORCH_CHECK(OH > 0 && OW > 0, "syrk_conv: empty output");
  const int64_t K = Cin * kh * kw;
  const int64_t D = K + (bias ? 1 : 0);
  const int64_t ldc = syrk_out_ld(C, D);
  const int64_t N = B * OH * OW;
  TORCH_CHECK(H < (1 << 30) && W < (1 << 30) && OH * OW < (1LL << 31));
  kfac::ConvGeom g{x.stride(0), x.stride(2), x.stride(3), (int32_t)H, (int32_t)W,
                   (int32_t)Cin, (int32_t)kw, (int32_t)sh, (int32_t)sw,
                   (int32_t)ph, (int32_t)pw, (int32_t)OH, (int32_t)OW};
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  int sp = splits > 0 ? (int)splits : (int)kfac::syrk_workspace_splits(N, D);
  at::Tensor ws = syrk_ws(C, D, sp);
  // fp32 input on the bf16x3 path: split it once into contiguous bf16 hi / lo
  // planes (stream-ordered temporary) so the SYRK loop converts nothing
  const int64_t elems = B * H * W * Cin;
  // (only for kernels with several taps: a 1x1 strided conv reads a
  // quarter of its input once, so splitting all of it costs more than the
  // in-loop split it saves)
  if (x.scalar_type() == at::kFloat && !fp32_exact && Cin % 8 == 0 && kh * kw > 1 &&
      N < (1LL << 24) && elems < (1LL << 29)) {
    at::Tensor planes = at::empty({2 * elems}, x.options().dtype(at::kBFloat16));
    kfac::syrk_split_planes(x.data_ptr<float>(), B, (int)H, (int)W, (int)Cin, x.stride(0),
                            x.stride(2), x.stride(3),
                            reinterpret_cast<uint16_t*>(planes.data_ptr()), cur_stream());
    kfac::ConvGeom gp{H * W * Cin, W * Cin, Cin, (int32_t)H, (int32_t)W, (int32_t)Cin,
                      (int32_t)kw, (int32_t)sh, (int32_t)sw, (int32_t)ph, (int32_t)pw,
                      (int32_t)OH, (int32_t)OW, elems, 0};
    kfac::syrk(kfac::kF32, planes.data_ptr(), N, K, /*ldx=*/K, bias, C.data_ptr<float>(), D,
               ldc, (float)alpha, (float)beta, sp, cur_stream(), &gp,
               ws.defined() ? ws.data_ptr<float>() : nullptr, syrk_ascale(ascale, C), false);
    return;
  }
  kfac::syrk(dtype_tag(x), x.data_ptr(), N, K, /*ldx=*/K, bias, C.data_ptr<float>(), D,
             ldc, (float)alpha, (float)beta, sp, cur_stream(), &g,
             ws.defined() ? ws.data_ptr<float>() : nullptr, syrk_ascale(ascale, C),
             fp32_exact);
}

// --------------------------------------------------------------- im2col
// x: [B, C, H, W] logical (any strides; NHWC fast path when channels_last).
// out: [B*OH*OW, ldo] rows; columns in (kh, kw, c) order for the NHWC path
// ("natural" order) and (c, kh, kw) order for the NCHW path (reference
// order, kfac/layers/modules.py:210-237).
void im2col(const at::Tensor& x, at::Tensor& out, int64_t kh, int64_t kw,
            int64_t sh, int64_t sw, int64_t ph, int64_t pw, bool natural) {
  check_cuda(x, "x");
  check_cuda(out, "out");
  TORCH_CHECK(x.dim() == 4, "x must be [B, C, H, W]");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1);
  const int64_t B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t OH = (H + 2 * ph - kh) / sh + 1;
  const int64_t OW = (W + 2 * pw - kw) / sw + 1;
  TORCH_CHECK(out.size(0) == B * OH * OW, "out rows");
  TORCH_CHECK(out.size(1) >= C * kh * kw, "out cols");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  if (natural) {
    TORCH_CHECK(x.stride(1) == 1, "natural im2col needs channels_last input");
    kfac::im2col_nhwc(dtype_tag(x), x.data_ptr(), B, H, W, C, x.stride(0),
                      x.stride(2), x.stride(3), (int)kh, (int)kw, (int)sh,
                      (int)sw, (int)ph, (int)pw, OH, OW, out.data_ptr(),
                      out.stride(0), dtype_tag(out), cur_stream());
  } else {
    kfac::im2col_nchw(dtype_tag(x), x.data_ptr(), B, C, H, W, x.stride(0),
                      x.stride(1), x.stride(2), x.stride(3), (int)kh, (int)kw,
                      (int)sh, (int)sw, (int)ph, (int)pw, OH, OW,
                      out.data_ptr(), out.stride(0), dtype_tag(out),
                      cur_stream());
  }
}

// ------------------------------------------------------------ precondition
void eigen_scale(at::Tensor& v, const c10::optional<at::Tensor>& dgda,
                 const c10::optional<at::Tensor>& dg,
                 const c10::optional<at::Tensor>& da, double damping) {
  check_cuda(v, "v");
  TORCH_CHECK(v.scalar_type() == at::kFloat && v.dim() == 2 &&
              v.stride(1) == 1);
  c10::hip::HIPGuardMasqueradingAsCUDA g(v.device());
  if (dgda.has_value()) {
    TORCH_CHECK(dgda->is_contiguous() && dgda->sizes() == v.sizes() &&
                dgda->scalar_type() == at::kFloat);
    kfac::eigen_scale(v.data_ptr<float>(), v.size(0), v.size(1), v.stride(0),
                      dgda->data_ptr<float>(), nullptr, nullptr, 0.f,
                      cur_stream());
  } else {
    TORCH_CHECK(dg.has_value() && da.has_value());
    TORCH_CHECK(dg->is_contiguous() && da->is_contiguous());
    TORCH_CHECK(dg->numel() == v.size(0) && da->numel() == v.size(1));
    kfac::eigen_scale(v.data_ptr<float>(), v.size(0), v.size(1), v.stride(0),
                      nullptr, dg->data_ptr<float>(), da->data_ptr<float>(),
                      (float)damping, cur_stream());
  }
}

// acc[0] += sum(P[:, :in] * Wg) + sum(P[:, in] * bg)   (double accumulator)
void kl_dot(const at::Tensor& p, const at::Tensor& wgrad,
            const c10::optional<at::Tensor>& bgrad, at::Tensor& acc) {
  check_cuda(p, "p");
  TORCH_CHECK(p.scalar_type() == at::kFloat && p.dim() == 2 &&
              p.stride(1) == 1);
  TORCH_CHECK(acc.scalar_type() == at::kDouble && acc.numel() >= 1);
  const int64_t rows = p.size(0);
  const int64_t wcols = p.size(1) - (bgrad.has_value() ? 1 : 0);
  TORCH_CHECK(wgrad.numel() == rows * wcols, "weight grad size");
  TORCH_CHECK(wgrad.is_contiguous(), "weight grad must be contiguous");
  c10::hip::HIPGuardMasqueradingAsCUDA g(p.device());
  const void* bptr = nullptr;
  int bdt = kfac::kF32;
  if (bgrad.has_value()) {
    TORCH_CHECK(bgrad->is_contiguous() && bgrad->numel() == rows);
    bptr = bgrad->data_ptr();
    bdt = dtype_tag(*bgrad);
  }
  kfac::kl_dot_accumulate(p.data_ptr<float>(), rows, p.size(1), p.stride(0),
                          wgrad.data_ptr(), dtype_tag(wgrad), wcols, bptr, bdt,
                          acc.data_ptr<double>(), cur_stream());
}

void kl_finalize(const at::Tensor& acc, at::Tensor& scale, double kl_clip,
                 double lr) {
  TORCH_CHECK(acc.scalar_type() == at::kDouble);
  TORCH_CHECK(scale.scalar_type() == at::kFloat);
  c10::hip::HIPGuardMasqueradingAsCUDA g(acc.device());
  kfac::kl_scale_finalize(acc.data_ptr<double>(), scale.data_ptr<float>(),
                          (float)kl_clip, (float)lr, cur_stream());
}

// wgrad = scale * P[:, :in], bgrad = scale * P[:, in]  (scale on device or
// None for 1)
void apply_grad(const at::Tensor& p, at::Tensor& wgrad,
                c10::optional<at::Tensor> bgrad,
                const c10::optional<at::Tensor>& scale) {
  check_cuda(p, "p");
  TORCH_CHECK(p.scalar_type() == at::kFloat && p.dim() == 2 &&
              p.stride(1) == 1);
  const int64_t rows = p.size(0);
  const int64_t wcols = p.size(1) - (bgrad.has_value() ? 1 : 0);
  TORCH_CHECK(wgrad.numel() == rows * wcols && wgrad.is_contiguous());
  c10::hip::HIPGuardMasqueradingAsCUDA g(p.device());
  void* bptr = nullptr;
  int bdt = kfac::kF32;
  if (bgrad.has_value()) {
    TORCH_CHECK(bgrad->is_contiguous() && bgrad->numel() == rows);
    bptr = bgrad->data_ptr();
    bdt = dtype_tag(*bgrad);
  }
  const float* sptr = nullptr;
  if (scale.has_value()) {
    TORCH_CHECK(scale->scalar_type() == at::kFloat);
    sptr = scale->data_ptr<float>();
  }
  kfac::apply_grad(p.data_ptr<float>(), rows, p.size(1), p.stride(0),
                   wgrad.data_ptr(), dtype_tag(wgrad), wcols, bptr, bdt, sptr,
                   cur_stream());
}

void fill_identity(at::Tensor& C) {
  check_cuda(C, "C");
  TORCH_CHECK(C.scalar_type() == at::kFloat && C.dim() == 2 &&
              C.size(0) == C.size(1) && C.stride(1) == 1);
  c10::hip::HIPGuardMasqueradingAsCUDA g(C.device());
  kfac::fill_identity_lerp(C.data_ptr<float>(), C.size(0), C.stride(0),
                           cur_stream());
}

// ------------------------------------------------------------ eigensolver
// A: [batch, n, n] fp32 symmetric.  Returns (evals [batch, n] ascending,
// evecs [batch, n, n] with eigenvectors in COLUMNS, like torch.linalg.eigh).
std::vector<at::Tensor> jacobi_eigh(const at::Tensor& A, int64_t max_sweeps,
                                    double tol) {
  check_cuda(A, "A");
  TORCH_CHECK(A.scalar_type() == at::kFloat && A.dim() == 3 &&
              A.size(1) == A.size(2) && A.is_contiguous());
  const int64_t batch = A.size(0), n = A.size(1);
  TORCH_CHECK(n <= kfac::jacobi_max_n(), "jacobi_eigh supports n <= ",
              kfac::jacobi_max_n());
  auto evals = at::empty({batch, n}, A.options());
  auto evecs = at::empty({batch, n, n}, A.options());
  c10::hip::HIPGuardMasqueradingAsCUDA g(A.device());
  if (batch > 0 && n > 0) {
    kfac::jacobi_eigh_batched(A.data_ptr<float>(), n, batch, n * n,
                              evals.data_ptr<float>(),
                              evecs.data_ptr<float>(), n * n,
                              (int)max_sweeps, (float)tol, cur_stream());
  }
  return {evals, evecs};
}

// ------------------------------------------------------- multi-tensor ops
// Build the device descriptor table for a list of layers.  Returns
// (table [uint8 on device], total_blocks).  The caller caches the table
// while the tensors' storages are unchanged.
// Upload a host-built descriptor table.  `host` is an optional pinned byte
// buffer owned by the caller (preallocated outside any HIP-graph capture);
// without it a pinned staging tensor is allocated here.
//
// Outside a capture the copy is a plain hipMemcpyAsync on the current stream.
// INSIDE a capture the table is allocated outside the graph's memory pool and
// no copy is recorded: the (device table, staging) pair is queued and
// flush_table_uploads() -- called by every capturing site right after its
// capture ends -- uploads it once, eagerly, before the graph's first replay.
// Round 2 allocated the table in the private pool and captured its copy: the
// pool hands a table's block to other tensors of the same graph, so the table
// was valid only from its copy node to its last reader within one replay --
// garbage when used eagerly (an illegal address for an eager step after a
// capture) and whenever graph work touching the recycled block ran between
// the copy and the readers (the post-refresh NaN of
// profiles/graph_replay_nonfinite_r2.txt; tools/graph_nan_probe.py,
// tools/graph_ptr_audit.py).
namespace {
std::mutex g_pending_mu;
std::vector<std::pair<at::Tensor, at::Tensor>> g_pending_uploads;

// Device twins of the caller's pinned staging slots (ops/precondition.py
// _TableCache): a table built inside a capture is written into the slot's
// persistent device buffer -- allocated eagerly, outside every graph pool --
// so a capture never allocates table memory.
std::mutex g_slot_mu;
std::unordered_map<const void*, at::Tensor> g_slot_dev;

bool current_stream_capturing() {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(cur_stream(), &st) != hipSuccess) return false;
  return st == hipStreamCaptureStatusActive;
}
}  // namespace

std::tuple<at::Tensor, at::Tensor> upload_table(
    const void* data, int64_t nbytes, const at::Device& device,
    const c10::optional<at::Tensor>& host) {
  at::Tensor cpu;
  if (host.has_value() && host->numel() >= nbytes) {
    cpu = *host;
    TORCH_CHECK(cpu.is_pinned() && cpu.scalar_type() == at::kByte && cpu.is_contiguous(),
                "table staging must be a pinned contiguous byte tensor");
  } else {
    cpu = at::empty({std::max<int64_t>(nbytes, 1)},
                    at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  }
  std::memcpy(cpu.data_ptr(), data, nbytes);
  const bool capturing = current_stream_capturing();
  at::Tensor dev_t;
  // Only a capture writes into the slot's persistent device twin.  An eager
  // upload gets a fresh stream-ordered allocation: the caller may launch the
  // table on another stream (it record_stream()s it at each launch), and a
  // recycled twin could be rewritten while such a launch is still queued.
  if (host.has_value() && capturing) {
    std::lock_guard<std::mutex> lk(g_slot_mu);
    auto it = g_slot_dev.find(host->data_ptr());
    if (it != g_slot_dev.end() && it->second.numel() >= std::max<int64_t>(nbytes, 1) &&
        it->second.device() == device)
      dev_t = it->second.narrow(0, 0, std::max<int64_t>(nbytes, 1));
  }
  if (!dev_t.defined()) {
    // NOT from a graph's private pool: the pool hands a block to other
    // tensors of the same graph, so a table there would be valid only from
    // its copy node to its last reader within one replay
    TORCH_CHECK(!capturing,
                "descriptor table built during a HIP-graph capture without a "
                "registered device slot (register_table_slot)");
    dev_t = at::empty({std::max<int64_t>(nbytes, 1)},
                      at::TensorOptions().dtype(at::kByte).device(device));
  }
  if (capturing) {
    std::lock_guard<std::mutex> lk(g_pending_mu);
    g_pending_uploads.emplace_back(dev_t.narrow(0, 0, std::max<int64_t>(nbytes, 1)),
                                   cpu.narrow(0, 0, std::max<int64_t>(nbytes, 1)));
  } else {
    C10_HIP_CHECK(hipMemcpyAsync(dev_t.data_ptr(), cpu.data_ptr(), nbytes,
                                 hipMemcpyHostToDevice, cur_stream()));
  }
  return {dev_t, cpu};
}

// Upload every table built inside the capture that just ended (on the
// current stream; the pinned-source copies record their stream events, so
// the staging is never recycled before they ran).  Returns the count.
void register_table_slot(const at::Tensor& host, const at::Tensor& dev) {
  TORCH_CHECK(host.is_pinned() && host.scalar_type() == at::kByte && dev.is_cuda() &&
                  dev.scalar_type() == at::kByte && dev.is_contiguous() &&
                  dev.numel() >= host.numel(),
              "register_table_slot: pinned byte host slot and a device byte buffer as large");
  std::lock_guard<std::mutex> lk(g_slot_mu);
  g_slot_dev[host.data_ptr()] = dev;
}

// Diagnostics (tools/graph_oop_audit.py): fill a raw device byte range that
// the caching allocator holds but has not handed out, to find graph nodes
// that read memory their graph does not own.
void memset_raw(int64_t addr, int64_t nbytes, int64_t value) {
  TORCH_CHECK(addr != 0 && nbytes >= 0, "memset_raw: bad range");
  C10_HIP_CHECK(hipMemsetAsync(reinterpret_cast<void*>(addr), static_cast<int>(value),
                               static_cast<size_t>(nbytes), cur_stream()));
}

void unregister_table_slot(const at::Tensor& host) {
  std::lock_guard<std::mutex> lk(g_slot_mu);
  g_slot_dev.erase(host.data_ptr());
}

int64_t flush_table_uploads() {
  std::vector<std::pair<at::Tensor, at::Tensor>> todo;
  {
    std::lock_guard<std::mutex> lk(g_pending_mu);
    todo.swap(g_pending_uploads);
  }
  TORCH_CHECK(todo.empty() || !current_stream_capturing(),
              "flush_table_uploads must run after the capture has ended");
  for (auto& p : todo) p.first.copy_(p.second, /*non_blocking=*/true);
  return (int64_t)todo.size();
}

// Returns (device table, block count, pinned host staging).  The host copy
// is returned so the caller keeps it alive: when the table is built inside a
// HIP-graph capture the H2D copy becomes a graph node that re-reads it on
// every replay.
std::tuple<at::Tensor, int64_t, at::Tensor> build_layer_table(
    const std::vector<at::Tensor>& ps, const std::vector<at::Tensor>& ws,
    const std::vector<c10::optional<at::Tensor>>& bs,
    const c10::optional<at::Tensor>& host_buf,
    const std::vector<double>& bscales) {
  TORCH_CHECK(ps.size() == ws.size() && ps.size() == bs.size());
  TORCH_CHECK(bscales.empty() || bscales.size() == ps.size(), "build_layer_table: bscales size");
  std::vector<kfac::LayerDesc> host(ps.size());
  int64_t blocks = 0;
  for (size_t i = 0; i < ps.size(); ++i) {
    const auto& p = ps[i];
    const auto& w = ws[i];
    check_cuda(p, "p");
    TORCH_CHECK(p.scalar_type() == at::kFloat && p.dim() == 2 &&
                p.stride(1) == 1);
    TORCH_CHECK(w.is_contiguous());
    const bool hb = bs[i].has_value();
    const int64_t rows = p.size(0), cols = p.size(1);
    const int64_t wcols = cols - (hb ? 1 : 0);
    TORCH_CHECK(w.numel() == rows * wcols, "layer ", i, ": weight grad size");
    TORCH_CHECK(rows * cols < (int64_t(1) << 31), "layer ", i, ": too many elements for the multi-tensor kernels");
    kfac::LayerDesc d{};
    d.p = p.data_ptr<float>();
    d.w = w.data_ptr();
    d.wdt = dtype_tag(w);
    d.b = nullptr;
    d.bdt = d.wdt;
    if (hb) {
      TORCH_CHECK(bs[i]->is_contiguous() && bs[i]->numel() == rows);
      d.b = bs[i]->data_ptr();
      d.bdt = dtype_tag(*bs[i]);
    }
    d.bscale = bscales.empty() ? 1.f : (float)bscales[i];
    d.rows = rows;
    d.cols = cols;
    d.ldp = p.stride(0);
    d.wcols = wcols;
    d.block_start = blocks;
    blocks += kfac::multi_blocks_for(rows, cols);
    host[i] = d;
  }
  const int64_t nbytes = (int64_t)(host.size() * sizeof(kfac::LayerDesc));
  at::Tensor dev_t, cpu;
  if (!ps.empty()) {
    std::tie(dev_t, cpu) = upload_table(host.data(), nbytes, ps[0].device(), host_buf);
  }
  return {dev_t, blocks, cpu};
}

// acc: >= total_blocks fp64 partial sums (one per block, no atomics)
void kl_dot_multi(const at::Tensor& table, int64_t nlayers,
                  int64_t total_blocks, at::Tensor& acc) {
  TORCH_CHECK(acc.scalar_type() == at::kDouble && acc.numel() >= total_blocks &&
                  acc.is_contiguous(),
              "kl_dot_multi: acc must hold one contiguous fp64 partial per block");
  c10::hip::HIPGuardMasqueradingAsCUDA g(acc.device());
  kfac::kl_dot_multi((const kfac::LayerDesc*)table.data_ptr(), (int)nlayers,
                     total_blocks, acc.data_ptr<double>(), cur_stream());
}

void kl_finalize_dev(const at::Tensor& acc, int64_t nparts, const at::Tensor& params,
                     at::Tensor& scale) {
  TORCH_CHECK(acc.scalar_type() == at::kDouble && acc.numel() >= nparts &&
              params.scalar_type() == at::kFloat &&
              scale.scalar_type() == at::kFloat);
  c10::hip::HIPGuardMasqueradingAsCUDA g(acc.device());
  kfac::kl_finalize_dev(acc.data_ptr<double>(), nparts, params.data_ptr<float>(),
                        scale.data_ptr<float>(), cur_stream());
}

// out[0] = fixed-order sum of acc[0:nparts] (one fp64 per-rank KL sum)
void kl_reduce_partials(const at::Tensor& acc, int64_t nparts, at::Tensor& out) {
  TORCH_CHECK(acc.scalar_type() == at::kDouble && acc.numel() >= nparts &&
              out.scalar_type() == at::kDouble && out.numel() >= 1);
  c10::hip::HIPGuardMasqueradingAsCUDA g(acc.device());
  kfac::kl_reduce_partials(acc.data_ptr<double>(), nparts, out.data_ptr<double>(),
                           cur_stream());
}

// ------------------------------------------------------- gemm3s (split images)
// A split image is a contiguous bf16 tensor [2, R, L]: plane 0 = hi, 1 = lo.
namespace {
int64_t ru(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

void check_image(const at::Tensor& t, const char* what) {
  check_cuda(t, what);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 && t.dim() == 3 && t.size(0) == 2 &&
                  t.is_contiguous(),
              what, ": split image must be a contiguous bf16 [2, R, L] tensor");
  TORCH_CHECK(t.size(2) % 8 == 0 && (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0,
              what, ": image rows must be 16-byte multiples, base 16-byte aligned");
}

// (rows, cols) the tile loads of one operand reach: k-contig [tile rows][K],
// m-contig [K][tile cols]
void check_extent(const at::Tensor& img, bool mc, int64_t mn, int64_t K, int64_t tile,
                  const char* what) {
  const int64_t R = img.size(1), L = img.size(2);
  const int64_t need_r = mc ? ru(K, 32) : ru(mn, tile);
  const int64_t need_l = mc ? ru(mn, tile) : ru(K, 32);
  TORCH_CHECK(R >= need_r && L >= need_l, what, ": image [", R, ", ", L,
              "] too small for the tile loads (needs [", need_r, ", ", need_l, "])");
}
}  // namespace

// Descriptor table of one grouped gemm3s launch; meta = (M, N, K) per GEMM.
// The K padding of every image (columns / rows K..ru(K, 32)) must be zero:
// images are allocated zeroed and only their logical part is ever written.
std::tuple<at::Tensor, int64_t, at::Tensor> build_gemm3s_table(
    const std::vector<at::Tensor>& As, const std::vector<at::Tensor>& Bs,
    const std::vector<at::Tensor>& Cs, const std::vector<c10::optional<at::Tensor>>& Ss,
    const std::vector<c10::optional<at::Tensor>>& dgs,
    const std::vector<c10::optional<at::Tensor>>& das, const std::vector<int64_t>& meta,
    const std::vector<double>& dampings, bool a_mc, bool b_mc, bool out_split,
    const c10::optional<at::Tensor>& host_buf) {
  const size_t n = As.size();
  TORCH_CHECK(Bs.size() == n && Cs.size() == n && Ss.size() == n && dgs.size() == n &&
                  das.size() == n && dampings.size() == n && meta.size() == 3 * n,
              "build_gemm3s_table: list sizes");
  const int64_t tm = kfac::gemm3s_tile_m(), tn = kfac::gemm3s_tile_n();
  std::vector<kfac::Gemm3sDesc> host(n);
  int tiles = 0;
  for (size_t i = 0; i < n; ++i) {
    const int64_t M = meta[3 * i], N = meta[3 * i + 1], K = meta[3 * i + 2];
    TORCH_CHECK(M > 0 && N > 0 && K > 0 && M < (1 << 30) && N < (1 << 30) && K < (1 << 30));
    check_image(As[i], "A");
    check_image(Bs[i], "B");
    check_extent(As[i], a_mc, M, K, tm, "A");
    check_extent(Bs[i], b_mc, N, K, tn, "B");
    kfac::Gemm3sDesc d{};
    d.A = (const uint16_t*)As[i].data_ptr();
    d.B = (const uint16_t*)Bs[i].data_ptr();
    d.a_plane = As[i].size(1) * As[i].size(2);
    d.b_plane = Bs[i].size(1) * Bs[i].size(2);
    d.lda = As[i].size(2);
    d.ldb = Bs[i].size(2);
    const auto& C = Cs[i];
    if (out_split) {
      check_image(C, "C");
      TORCH_CHECK(C.size(1) >= M && C.size(2) >= N, "C image too small");
      d.c_plane = C.size(1) * C.size(2);
      d.ldc = C.size(2);
    } else {
      check_cuda(C, "C");
      TORCH_CHECK(C.scalar_type() == at::kFloat && C.dim() == 2 && C.stride(1) == 1 &&
                      C.size(0) >= M && C.size(1) >= N,
                  "fp32 C must be [>= M, >= N] with unit column stride");
      d.c_plane = 0;
      d.ldc = C.stride(0);
    }
    d.C = C.data_ptr();
    d.S = nullptr;
    d.lds = 0;
    if (Ss[i].has_value() && Ss[i]->defined()) {
      const auto& S = *Ss[i];
      TORCH_CHECK(S.scalar_type() == at::kFloat && S.dim() == 2 && S.stride(1) == 1 &&
                      S.size(0) >= M && S.size(1) >= N,
                  "S must be fp32 [>= M, >= N] with unit column stride");
      d.S = S.data_ptr<float>();
      d.lds = S.stride(0);
    }
    d.dg = d.da = nullptr;
    if (dgs[i].has_value() && dgs[i]->defined()) {
      TORCH_CHECK(das[i].has_value() && das[i]->defined(), "dg needs da");
      TORCH_CHECK(dgs[i]->scalar_type() == at::kFloat && dgs[i]->is_contiguous() &&
                      dgs[i]->numel() >= M && das[i]->scalar_type() == at::kFloat &&
                      das[i]->is_contiguous() && das[i]->numel() >= N,
                  "dg / da must be contiguous fp32 vectors of length >= M / N");
      d.dg = dgs[i]->data_ptr<float>();
      d.da = das[i]->data_ptr<float>();
    }
    d.damping = (float)dampings[i];
    d.M = (int32_t)M;
    d.N = (int32_t)N;
    d.K = (int32_t)K;
    d.tiles_n = (int32_t)((N + tn - 1) / tn);
    d.tile_start = tiles;
    tiles += (int)((M + tm - 1) / tm) * d.tiles_n;
    host[i] = d;
  }
  const int64_t nbytes = (int64_t)(n * sizeof(kfac::Gemm3sDesc));
  at::Tensor dev_t, cpu;
  if (n > 0) std::tie(dev_t, cpu) = upload_table(host.data(), nbytes, As[0].device(), host_buf);
  return {dev_t, tiles, cpu};
}

void gemm3s_grouped(const at::Tensor& table, int64_t n, int64_t tiles, bool a_mc, bool b_mc,
                    bool out_split) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(table.device());
  kfac::gemm3s_grouped((const kfac::Gemm3sDesc*)table.data_ptr(), (int)n, (int)tiles, a_mc,
                       b_mc, out_split, cur_stream());
}

// fp32 [rows][cols] (+ extra column from a vector) -> split images
std::tuple<at::Tensor, int64_t, at::Tensor> build_split_table(
    const std::vector<at::Tensor>& srcs, const std::vector<c10::optional<at::Tensor>>& extras,
    const std::vector<at::Tensor>& dsts, const c10::optional<at::Tensor>& host_buf) {
  const size_t n = srcs.size();
  TORCH_CHECK(extras.size() == n && dsts.size() == n, "build_split_table: list sizes");
  std::vector<kfac::SplitDesc> host(n);
  int64_t blocks = 0;
  for (size_t i = 0; i < n; ++i) {
    const auto& x = srcs[i];
    check_cuda(x, "src");
    TORCH_CHECK(x.scalar_type() == at::kFloat && x.dim() == 2 && x.stride(1) == 1,
                "split source must be fp32 2-D with unit column stride");
    check_image(dsts[i], "dst");
    const bool ex = extras[i].has_value() && extras[i]->defined();
    const int64_t rows = x.size(0), cols = x.size(1), tot = cols + (ex ? 1 : 0);
    TORCH_CHECK(dsts[i].size(1) >= rows && dsts[i].size(2) >= ru(tot, 4),
                "split image too small for its source");
    if (ex) {
      TORCH_CHECK(extras[i]->scalar_type() == at::kFloat && extras[i]->is_contiguous() &&
                      extras[i]->numel() == rows,
                  "extra column must be a contiguous fp32 vector of length rows");
    }
    kfac::SplitDesc d{};
    d.src = x.data_ptr<float>();
    d.extra = ex ? extras[i]->data_ptr<float>() : nullptr;
    d.dst = (uint16_t*)dsts[i].data_ptr();
    d.lds = x.stride(0);
    d.ldd = dsts[i].size(2);
    d.plane = dsts[i].size(1) * dsts[i].size(2);
    d.rows = (int32_t)rows;
    d.cols = (int32_t)cols;
    d.vec = (x.stride(0) % 4 == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0) ? 1 : 0;
    d.block_start = blocks;
    blocks += kfac::split_blocks_for(rows, tot);
    host[i] = d;
  }
  const int64_t nbytes = (int64_t)(n * sizeof(kfac::SplitDesc));
  at::Tensor dev_t, cpu;
  if (n > 0) std::tie(dev_t, cpu) = upload_table(host.data(), nbytes, srcs[0].device(), host_buf);
  return {dev_t, blocks, cpu};
}

// Multi-tensor cast table: srcs[i] (fp32 or bf16) -> dsts[i] (the other
// dtype), element by element in STORAGE order, so the pairs must share shape
// and strides and be dense (non-overlapping, no gaps).
std::tuple<at::Tensor, int64_t, at::Tensor> build_cast_table(
    const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts,
    const c10::optional<at::Tensor>& host_buf) {
  const size_t n = srcs.size();
  TORCH_CHECK(dsts.size() == n, "build_cast_table: list sizes");
  std::vector<kfac::CastDesc> host(n);
  int64_t blocks = 0;
  for (size_t i = 0; i < n; ++i) {
    const auto& x = srcs[i];
    const auto& y = dsts[i];
    check_cuda(x, "src");
    check_cuda(y, "dst");
    const bool f2b = x.scalar_type() == at::kFloat && y.scalar_type() == at::kBFloat16;
    const bool b2f = x.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kFloat;
    TORCH_CHECK(f2b || b2f, "cast pairs must be fp32 -> bf16 or bf16 -> fp32");
    TORCH_CHECK(i == 0 || (f2b == (srcs[0].scalar_type() == at::kFloat)),
                "one cast direction per table");
    TORCH_CHECK(x.sizes() == y.sizes() && x.strides() == y.strides(),
                "cast pair ", i, ": shapes and strides must match");
    TORCH_CHECK(x.is_non_overlapping_and_dense(), "cast pair ", i, ": source must be dense");
    kfac::CastDesc d{};
    d.src = x.data_ptr();
    d.dst = y.data_ptr();
    d.n = x.numel();
    d.vec = ((reinterpret_cast<uintptr_t>(x.data_ptr()) | reinterpret_cast<uintptr_t>(y.data_ptr())) & 15) == 0;
    d.block_start = blocks;
    blocks += kfac::cast_blocks_for(d.n);
    host[i] = d;
  }
  const int64_t nbytes = (int64_t)(n * sizeof(kfac::CastDesc));
  at::Tensor dev_t, cpu;
  if (n > 0) std::tie(dev_t, cpu) = upload_table(host.data(), nbytes, srcs[0].device(), host_buf);
  return {dev_t, blocks, cpu};
}

void cast_multi(const at::Tensor& table, int64_t n, int64_t blocks, bool to_bf16) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(table.device());
  kfac::cast_multi((const kfac::CastDesc*)table.data_ptr(), (int)n, blocks, to_bf16, cur_stream());
}

void split_pad_multi(const at::Tensor& table, int64_t n, int64_t blocks) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(table.device());
  kfac::split_pad_multi((const kfac::SplitDesc*)table.data_ptr(), (int)n, blocks, cur_stream());
}

void apply_multi(const at::Tensor& table, int64_t nlayers,
                 int64_t total_blocks, const c10::optional<at::Tensor>& scale) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(table.device());
  kfac::apply_multi((const kfac::LayerDesc*)table.data_ptr(), (int)nlayers,
                    total_blocks,
                    scale.has_value() ? scale->data_ptr<float>() : nullptr,
                    cur_stream());
}

const float* opt_ptr(const c10::optional<at::Tensor>& t, int64_t numel,
                     const char* what) {
  if (!t.has_value()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() &&
                  t->numel() == numel,
              what, ": expected a contiguous fp32 tensor of ", numel, " elements");
  return t->data_ptr<float>();
}

bool vec_ok(const at::Tensor& t) {
  return (t.stride(0) % 4 == 0) &&
         ((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0);
}

// Grouped bf16x3 GEMM table.  For layer i (logical C = A . B, [M,N,K]):
//   a_kc: As[i] is [M, Kmain] (+ optional A_extra column -> K = Kmain + 1),
//   else As[i] is the stored [K, M] (logical A = As^T);
//   b_kc: Bs[i] is the stored [N, K] (logical B = Bs^T), else [K, N].
// Optional epilogue scale: Ss[i] [M, N] or dgs[i] [M] with das[i] [N].
// Layers are sorted by K (descending) so long tiles are dispatched first.
// Returns (device table, tile count, pinned host staging) -- see
// build_layer_table for why the host copy is returned.
std::tuple<at::Tensor, int64_t, at::Tensor> build_gemm_table(
    const std::vector<at::Tensor>& As,
    const std::vector<c10::optional<at::Tensor>>& A_extras,
    const std::vector<at::Tensor>& Bs, const std::vector<at::Tensor>& Cs,
    const std::vector<c10::optional<at::Tensor>>& Ss,
    const std::vector<c10::optional<at::Tensor>>& dgs,
    const std::vector<c10::optional<at::Tensor>>& das,
    const std::vector<double>& dampings, bool a_kc, bool b_kc,
    const c10::optional<at::Tensor>& host_buf,
    const std::vector<c10::optional<at::Tensor>>& A_hls,
    const std::vector<c10::optional<at::Tensor>>& B_hls) {
  const size_t n = As.size();
  TORCH_CHECK(A_extras.size() == n && Bs.size() == n && Cs.size() == n &&
              Ss.size() == n && dgs.size() == n && das.size() == n &&
              dampings.size() == n);
  TORCH_CHECK(A_hls.empty() || A_hls.size() == n, "gemm3: A_hls size");
  TORCH_CHECK(B_hls.empty() || B_hls.size() == n, "gemm3: B_hls size");
  // pre-split operand: [rows, cols / 4, 8] bf16 (hi x4, lo x4 per group of
  // 4 elements) matching a contiguous fp32 operand with cols % 4 == 0
  auto hl = [](const c10::optional<at::Tensor>& t, const at::Tensor& op,
               const uint16_t** h) {
    *h = nullptr;
    if (!t.has_value() || !t->defined()) return;
    check_cuda(*t, "pre-split operand");
    TORCH_CHECK(op.is_contiguous() && op.size(1) % 4 == 0,
                "gemm3: pre-split needs a contiguous fp32 operand with cols % 4 == 0");
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->dim() == 3 && t->is_contiguous() &&
                    t->size(0) == op.size(0) && t->size(1) == op.size(1) / 4 &&
                    t->size(2) == 8 && (reinterpret_cast<uintptr_t>(t->data_ptr()) % 16) == 0,
                "gemm3: pre-split operand must be a contiguous [rows, cols/4, 8] bf16 tensor");
    *h = reinterpret_cast<const uint16_t*>(t->data_ptr());
  };
  std::vector<kfac::GemmDesc> host(n);
  for (size_t i = 0; i < n; ++i) {
    const auto& A = As[i];
    const auto& B = Bs[i];
    const auto& C = Cs[i];
    for (const at::Tensor* t : {&A, &B, &C}) {
      check_cuda(*t, "gemm operand");
      TORCH_CHECK(t->scalar_type() == at::kFloat && t->dim() == 2 &&
                      (t->stride(1) == 1 || t->size(1) == 1),
                  "gemm3: operands must be fp32 2-D with unit column stride");
    }
    const int64_t M = C.size(0), N = C.size(1);
    const bool extra = A_extras[i].has_value();
    TORCH_CHECK(!extra || a_kc, "gemm3: an extra A column needs a k-contiguous A");
    const int64_t Kmain = a_kc ? A.size(1) : A.size(0);
    const int64_t K = Kmain + (extra ? 1 : 0);
    TORCH_CHECK((a_kc ? A.size(0) : A.size(1)) == M, "gemm3 layer ", i, ": A shape");
    TORCH_CHECK(b_kc ? (B.size(0) == N && B.size(1) == K) : (B.size(0) == K && B.size(1) == N),
                "gemm3 layer ", i, ": B shape");
    TORCH_CHECK(M < (1 << 30) && N < (1 << 30) && K < (1 << 30));
    kfac::GemmDesc d{};
    d.A = A.data_ptr<float>();
    d.A_extra = opt_ptr(A_extras[i], M, "A_extra");
    d.B = B.data_ptr<float>();
    d.C = C.data_ptr<float>();
    d.lda = A.stride(0);
    d.ldb = B.stride(0);
    d.ldc = C.stride(0);
    d.S = nullptr;
    d.lds = 0;
    if (Ss[i].has_value()) {
      const auto& S = *Ss[i];
      TORCH_CHECK(S.scalar_type() == at::kFloat && S.dim() == 2 && S.size(0) == M &&
                  S.size(1) == N && (S.stride(1) == 1 || N == 1), "gemm3: S shape");
      d.S = S.data_ptr<float>();
      d.lds = S.stride(0);
    }
    d.dg = opt_ptr(dgs[i], M, "dg");
    d.da = opt_ptr(das[i], N, "da");
    TORCH_CHECK((d.dg == nullptr) == (d.da == nullptr), "gemm3: dg and da go together");
    d.M = (int32_t)M;
    d.N = (int32_t)N;
    d.K = (int32_t)K;
    d.Kmain = (int32_t)Kmain;
    d.tiles_n = (int32_t)((N + 127) / 128);
    d.damping = (float)dampings[i];
    if (!A_hls.empty()) {
      hl(A_hls[i], A, &d.Ah);
      TORCH_CHECK(d.Ah == nullptr || !extra, "gemm3: pre-split A cannot carry an extra column");
    }
    if (!B_hls.empty()) hl(B_hls[i], B, &d.Bh);
    d.vec = (vec_ok(A) ? 1 : 0) | (vec_ok(B) ? 2 : 0);
    host[i] = d;
  }
  std::stable_sort(host.begin(), host.end(),
                   [](const kfac::GemmDesc& x, const kfac::GemmDesc& y) { return x.K > y.K; });
  int64_t tiles = 0;
  for (auto& d : host) {
    d.tile_start = (int32_t)tiles;
    tiles += (int64_t)((d.M + 127) / 128) * d.tiles_n;
  }
  TORCH_CHECK(tiles < (1LL << 30));
  at::Tensor dev_t, cpu;
  if (n > 0) {
    const int64_t nbytes = (int64_t)(n * sizeof(kfac::GemmDesc));
    std::tie(dev_t, cpu) = upload_table(host.data(), nbytes, Cs[0].device(), host_buf);
  }
  return {dev_t, tiles, cpu};
}

// The split count gemm3_single actually uses for a K-long reduction asked
// for `want` splits: equal whole-k-tile shares, none empty.
int64_t gemm3_mm_splits_for(int64_t K, int64_t want) {
  const int64_t kts = (K + 31) / 32;
  int64_t sp = want < 1 ? 1 : (want > kts ? kts : want);
  const int64_t per = (kts + sp - 1) / sp;
  return (kts + per - 1) / per;
}

// the BN statistics partials a single-pass gemm3 GEMM writes for an
// [M, N] output (GemmDesc::bnpart): fp32 [2 * ceil(M / 128)][2][N]
static float* bn_part_ptr(const c10::optional<at::Tensor>& p, int64_t M, int64_t N,
                          const at::Device& dev) {
  if (!p.has_value() || !p->defined()) return nullptr;
  check_cuda(*p, "bnpart");
  TORCH_CHECK(p->device() == dev && p->scalar_type() == at::kFloat && p->is_contiguous() &&
                  p->numel() == 2 * ((M + 127) / 128) * 2 * N,
              "bnpart: contiguous fp32 [2 * ceil(M / 128)][2][N]");
  return p->data_ptr<float>();
}

// One fp32 GEMM C[M,N] = A . B on bf16x3 MFMA (csrc/gemm3.hip), the
// descriptor passed by value (no table upload: capturable as a single
// kernel node).  a_kc: A is [M, K], else the stored [K, M]; b_kc: B is the
// stored [N, K], else [K, N].  C is overwritten.  splits > 1: split-K, C is
// [splits, M, N] and receives one partial product per split (the caller
// sums them; k-tiles are shared out equally, see gemm3_mm_splits).
void gemm3_mm(const at::Tensor& A, const at::Tensor& B, const at::Tensor& C, bool a_kc,
              bool b_kc, int64_t splits, const c10::optional<at::Tensor>& bnpart,
              const c10::optional<at::Tensor>& addend) {
  TORCH_CHECK(splits >= 1, "gemm3_mm: splits >= 1");
  if (splits > 1) {
    check_cuda(C, "gemm3_mm partials");
    TORCH_CHECK(C.dim() == 3 && C.size(0) == splits && C.is_contiguous() &&
                    C.scalar_type() == at::kFloat,
                "gemm3_mm: split-K output must be a contiguous fp32 [splits, M, N]");
    const int64_t kk = a_kc ? A.size(1) : A.size(0);
    TORCH_CHECK(splits == gemm3_mm_splits_for(kk, splits),
                "gemm3_mm: splits must come from gemm3_mm_splits");
  }
  const at::Tensor C2 = splits > 1 ? C[0] : C;
  for (const at::Tensor* t : {&A, &B, &C2}) {
    check_cuda(*t, "gemm3_mm operand");
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->dim() == 2 && t->stride(1) == 1,
                "gemm3_mm: operands must be fp32 2-D with unit column stride");
  }
  TORCH_CHECK(A.device() == B.device() && A.device() == C.device(), "gemm3_mm: one device");
  const int64_t M = C2.size(0), N = C2.size(1);
  const int64_t K = a_kc ? A.size(1) : A.size(0);
  TORCH_CHECK((a_kc ? A.size(0) : A.size(1)) == M, "gemm3_mm: A shape");
  TORCH_CHECK(b_kc ? (B.size(0) == N && B.size(1) == K) : (B.size(0) == K && B.size(1) == N),
              "gemm3_mm: B shape");
  TORCH_CHECK(M < (1 << 30) && N < (1 << 30) && K < (1 << 30), "gemm3_mm: too large");
  kfac::GemmDesc d{};
  d.A = A.data_ptr<float>();
  d.B = B.data_ptr<float>();
  d.C = C2.data_ptr<float>();
  d.lda = A.stride(0);
  d.ldb = B.stride(0);
  d.ldc = C2.stride(0);
  d.M = (int32_t)M;
  d.N = (int32_t)N;
  d.K = (int32_t)K;
  d.Kmain = (int32_t)K;
  d.tiles_n = (int32_t)((N + 127) / 128);
  d.vec = (vec_ok(A) ? 1 : 0) | (vec_ok(B) ? 2 : 0);
  d.bnpart = bn_part_ptr(bnpart, M, N, C.device());
  TORCH_CHECK(d.bnpart == nullptr || splits == 1, "gemm3_mm: bnpart needs splits == 1");
  if (addend.has_value() && addend->defined()) {
    // C = A . B + addend (addend may be C itself)
    check_cuda(*addend, "gemm3_mm addend");
    TORCH_CHECK(splits == 1 && addend->scalar_type() == at::kFloat && addend->dim() == 2 &&
                    addend->size(0) == M && addend->size(1) == N && addend->stride(1) == 1 &&
                    addend->stride(0) == C2.stride(0) && addend->device() == C.device(),
                "gemm3_mm: addend must be an fp32 [M, N] with C's strides (splits == 1)");
    d.D = addend->data_ptr<float>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(C.device());
  if (K == 0) {
    if (d.D != nullptr) {
      if (addend->data_ptr() != C.data_ptr()) C.copy_(*addend);
    } else {
      C.zero_();
    }
    return;
  }
  kfac::gemm3_single(d, a_kc, b_kc, (int)splits, M * N, cur_stream());
}


// Implicit-GEMM convolution on bf16x3 MFMA (csrc/gemm3.hip): x [N, C, H, W]
// and w [Cout, C, kh, kw] both channels_last fp32, C % 4 == 0 (% 32 with
// flipw), no dilation or groups; returns y [N, Cout, Ho, Wo] channels_last.
// flipw: w is a stride-1 forward weight [Cf, Cout, kh, kw] (Cf = x's C) and
// the convolution applied is its flipped transpose -- the input gradient of
// that convolution when x is dy (pad = kh - 1 - forward pad).
at::Tensor sum_splits(const at::Tensor& part, const c10::optional<at::Tensor>& out_opt);

at::Tensor gemm3_conv(const at::Tensor& x, const at::Tensor& w, int64_t stride, int64_t pad,
                      bool flipw, const c10::optional<at::Tensor>& bnpart) {
  check_cuda(x, "gemm3_conv x");
  check_cuda(w, "gemm3_conv w");
  TORCH_CHECK(x.scalar_type() == at::kFloat && w.scalar_type() == at::kFloat && x.dim() == 4 &&
                  w.dim() == 4, "gemm3_conv: fp32 4-D operands");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "gemm3_conv: channels_last operands");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Co = flipw ? w.size(1) : w.size(0), kh = w.size(2), kw = w.size(3);
  TORCH_CHECK((flipw ? w.size(0) : w.size(1)) == C && C % 4 == 0 && (!flipw || C % 32 == 0),
              "gemm3_conv: C must match and be a multiple of 4 (32 with flipw)");
  TORCH_CHECK(!flipw || (stride == 1 && Co % 4 == 0), "gemm3_conv: flipw needs stride 1");
  TORCH_CHECK(stride >= 1 && pad >= 0 && kh >= 1 && kw >= 1, "gemm3_conv: geometry");
  const int64_t Ho = (H + 2 * pad - kh) / stride + 1, Wo = (W + 2 * pad - kw) / stride + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "gemm3_conv: empty output");
  TORCH_CHECK(N * H * W * C < (1LL << 31) && N * Ho * Wo < (1LL << 30) && kh * kw * C < (1 << 30),
              "gemm3_conv: too large");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(w.data_ptr()) & 15) == 0,
              "gemm3_conv: 16-byte aligned operands");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto y = at::empty({N, Co, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int sp = kfac::gemm3_conv_splits((int)N, (int)H, (int)W, (int)C, (int)Co, (int)kh,
                                         (int)kw, (int)stride, (int)pad);
  // split-K partials summed in fixed order by one reduction (deterministic)
  at::Tensor part = sp > 1 ? at::empty({sp, N * Ho * Wo, Co}, x.options()) : y;
  // BN statistics only from a single pass (the caller checks
  // gemm3_conv_splits first); a split launch leaves bnpart unwritten
  float* bnp = bn_part_ptr(bnpart, N * Ho * Wo, Co, x.device());
  TORCH_CHECK(bnp == nullptr || (sp == 1 && !flipw), "gemm3_conv: bnpart needs a single pass");
  kfac::gemm3_conv(x.data_ptr<float>(), w.data_ptr<float>(), part.data_ptr<float>(), (int)N,
                   (int)H, (int)W, (int)C, (int)Co, (int)kh, (int)kw, (int)stride, (int)pad, sp,
                   flipw, cur_stream(), bnp);
  if (sp > 1) sum_splits(part, y.permute({0, 2, 3, 1}).view({N * Ho * Wo, Co}));
  return y;
}

// Weight gradient of gemm3_conv: x [N, C, H, W] and dy [N, Cout, Ho, Wo]
// channels_last fp32 (C % 4 == 0, Cout % 4 == 0); returns dw [Cout, C, kh,
// kw] channels_last (split-K partials summed in fixed order).
at::Tensor gemm3_conv_wgrad(const at::Tensor& x, const at::Tensor& dy, int64_t kh, int64_t kw,
                            int64_t stride, int64_t pad) {
  check_cuda(x, "gemm3_conv_wgrad x");
  check_cuda(dy, "gemm3_conv_wgrad dy");
  TORCH_CHECK(x.scalar_type() == at::kFloat && dy.scalar_type() == at::kFloat && x.dim() == 4 &&
                  dy.dim() == 4, "gemm3_conv_wgrad: fp32 4-D operands");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "gemm3_conv_wgrad: channels_last operands");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Co = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  TORCH_CHECK(dy.size(0) == N && Ho == (H + 2 * pad - kh) / stride + 1 &&
                  Wo == (W + 2 * pad - kw) / stride + 1, "gemm3_conv_wgrad: geometry");
  TORCH_CHECK(C % 4 == 0 && Co % 4 == 0, "gemm3_conv_wgrad: channels must be multiples of 4");
  TORCH_CHECK(N * Ho * Wo < (1 << 22) && N * H * W * C < (1LL << 31),
              "gemm3_conv_wgrad: too large");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  const int sp = kfac::gemm3_wgrad_splits((int)(N * Ho * Wo), (int)Co, (int)(kh * kw * C));
  auto part = at::empty({sp, Co, kh * kw * C}, x.options());
  kfac::gemm3_conv_wgrad(x.data_ptr<float>(), dy.data_ptr<float>(), part.data_ptr<float>(),
                         (int)N, (int)H, (int)W, (int)C, (int)Co, (int)kh, (int)kw, (int)stride,
                         (int)pad, sp, cur_stream());
  auto dw = sp > 1 ? sum_splits(part, c10::nullopt) : part[0];
  return dw.view({Co, kh, kw, C}).permute({0, 3, 1, 2});
}

// x[:, :, ::sh, ::sw] of a channels_last fp32 tensor (C % 4 == 0), and the
// adjoint: the gradient scattered to every kept pixel of a zero tensor of
// the input's shape (csrc/subsample.hip)
static void check_nhwc4(const at::Tensor& t, const char* what) {
  check_cuda(t, what);
  TORCH_CHECK(t.scalar_type() == at::kFloat && t.dim() == 4 &&
                  t.is_contiguous(at::MemoryFormat::ChannelsLast) && t.size(1) % 4 == 0 &&
                  (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0,
              what, ": expected a 16-byte aligned channels_last fp32 tensor with C % 4 == 0");
}

// out = part.sum(0) for a contiguous fp32 [S, ...] partial stack (split-K);
// `out` contiguous with part[0]'s element count, or undefined (allocated)
at::Tensor sum_splits(const at::Tensor& part, const c10::optional<at::Tensor>& out_opt) {
  check_cuda(part, "sum_splits partials");
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() >= 2,
              "sum_splits: contiguous fp32 [S, ...] partials");
  const int64_t S = part.size(0), T = part.numel() / (S > 0 ? S : 1);
  at::Tensor out = out_opt.has_value() ? *out_opt : at::empty(part.sizes().slice(1), part.options());
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == T,
              "sum_splits: output must be contiguous fp32 with one partial's elements");
  const bool vec = T % 4 == 0 && (reinterpret_cast<uintptr_t>(part.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(out.data_ptr()) & 15) == 0;
  if (!vec) {
    auto flat = out.view({T});
    at::sum_out(flat, part.view({S, T}), {0});
    return out;
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(part.device());
  kfac::sum_splits(part.data_ptr<float>(), out.data_ptr<float>(), (int)S, T, cur_stream());
  return out;
}

at::Tensor subsample_fwd(const at::Tensor& x, int64_t sh, int64_t sw) {
  check_nhwc4(x, "subsample x");
  TORCH_CHECK(sh >= 1 && sw >= 1, "subsample: strides");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  auto y = at::empty({N, C, (H + sh - 1) / sh, (W + sw - 1) / sw},
                     x.options().memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  kfac::subsample_fwd(x.data_ptr<float>(), y.data_ptr<float>(), (int)N, (int)H, (int)W, (int)C,
                      (int)sh, (int)sw, cur_stream());
  return y;
}

at::Tensor subsample_bwd(const at::Tensor& gy, int64_t H, int64_t W, int64_t sh, int64_t sw) {
  check_nhwc4(gy, "subsample gradient");
  const int64_t N = gy.size(0), C = gy.size(1);
  TORCH_CHECK(gy.size(2) == (H + sh - 1) / sh && gy.size(3) == (W + sw - 1) / sw,
              "subsample_bwd: gradient shape");
  auto gx = at::empty({N, C, H, W}, gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuardMasqueradingAsCUDA g(gy.device());
  kfac::subsample_bwd(gy.data_ptr<float>(), gx.data_ptr<float>(), (int)N, (int)H, (int)W, (int)C,
                      (int)sh, (int)sw, cur_stream());
  return gx;
}

// [N, C, H, W] channels_last fp32 -> [N, ceil4(C), H, W] channels_last,
// the extra channels zero (csrc/subsample.hip pad_channels4)
at::Tensor pad_channels4(const at::Tensor& x) {
  check_cuda(x, "pad_channels4 input");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "pad_channels4: channels_last fp32 [N, C, H, W]");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t C4 = (C + 3) / 4 * 4;
  auto y = at::empty({N, C4, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  kfac::pad_channels4(x.data_ptr<float>(), y.data_ptr<float>(), N * H * W, (int)C, cur_stream());
  return y;
}

// gx += adjoint(gy), in place: gx is the other branch's full-size gradient
void subsample_bwd_acc(const at::Tensor& gy, const at::Tensor& gx, int64_t sh, int64_t sw) {
  check_nhwc4(gy, "subsample gradient");
  check_nhwc4(gx, "subsample accumulation target");
  const int64_t N = gy.size(0), C = gy.size(1), H = gx.size(2), W = gx.size(3);
  TORCH_CHECK(gx.size(0) == N && gx.size(1) == C && gy.size(2) == (H + sh - 1) / sh &&
                  gy.size(3) == (W + sw - 1) / sw && gx.device() == gy.device(),
              "subsample_bwd_acc: shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(gy.device());
  kfac::subsample_bwd_acc(gy.data_ptr<float>(), gx.data_ptr<float>(), (int)N, (int)H, (int)W,
                          (int)C, (int)sh, (int)sw, cur_stream());
}

// gx[B, C, H, W] (channels_last, cols' dtype) = col2im(cols): the adjoint of
// the NHWC im2col, cols the contiguous fp32 or bf16 [B * OH * OW, kh * kw * C]
// in (ky, kx, c) column order (csrc/im2col.hip col2im_nhwc; fixed-order fp32
// sums)
at::Tensor col2im_nhwc(const at::Tensor& cols, int64_t B, int64_t C, int64_t H, int64_t W,
                       int64_t kh, int64_t kw, int64_t stride, int64_t pad) {
  check_cuda(cols, "col2im cols");
  const bool bf = cols.scalar_type() == at::kBFloat16;
  TORCH_CHECK((bf ? C % 8 : C % 4) == 0 && kh >= 1 && kw >= 1 && stride >= 1 && pad >= 0,
              "col2im_nhwc: C % 4 == 0 (fp32) / C % 8 == 0 (bf16), positive geometry");
  const int64_t OH = (H + 2 * pad - kh) / stride + 1, OW = (W + 2 * pad - kw) / stride + 1;
  TORCH_CHECK(OH >= 1 && OW >= 1 && (bf || cols.scalar_type() == at::kFloat) && cols.dim() == 2 &&
                  cols.is_contiguous() && cols.size(0) == B * OH * OW &&
                  cols.size(1) == kh * kw * C &&
                  (reinterpret_cast<uintptr_t>(cols.data_ptr()) & 15) == 0,
              "col2im_nhwc: cols must be a 16-byte aligned contiguous fp32 / bf16 [B*OH*OW, kh*kw*C]");
  TORCH_CHECK(B * H * W * C < ((int64_t)1 << 31) * 4 && B * H * W < ((int64_t)1 << 31),
              "col2im_nhwc: too large");
  auto gx = at::empty({B, C, H, W}, cols.options().memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuardMasqueradingAsCUDA g(cols.device());
  kfac::col2im_nhwc(bf ? kfac::kBF16 : kfac::kF32, cols.data_ptr(), gx.data_ptr(), (int)B, (int)H,
                    (int)W, (int)C, (int)OH, (int)OW, (int)kh, (int)kw, (int)stride, (int)stride,
                    (int)pad, (int)pad, cur_stream());
  return gx;
}

// max_pool2d of a channels_last fp32 (C % 4 == 0) / bf16 (C % 8 == 0)
// tensor (square kernel k, stride s, padding p, dilation 1, floor mode):
// returns (y, code) with code the uint8 [N, OH, OW, C] window position of
// each maximum (csrc/pool.hip)
static void check_pool_input(const at::Tensor& t, const char* what) {
  check_cuda(t, what);
  const bool bf = t.scalar_type() == at::kBFloat16;
  TORCH_CHECK((bf || t.scalar_type() == at::kFloat) && t.dim() == 4 &&
                  t.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  t.size(1) % (bf ? 8 : 4) == 0 &&
                  (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0,
              what, ": 16-byte aligned channels_last fp32 (C % 4 == 0) or bf16 (C % 8 == 0)");
}

std::vector<at::Tensor> maxpool_nhwc_fwd(const at::Tensor& x, int64_t k, int64_t s, int64_t p) {
  check_pool_input(x, "maxpool input");
  TORCH_CHECK(k >= 1 && k <= 15 && s >= 1 && p >= 0 && 2 * p <= k, "maxpool: geometry");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t OH = (H + 2 * p - k) / s + 1, OW = (W + 2 * p - k) / s + 1;
  TORCH_CHECK(OH >= 1 && OW >= 1 && N * H * W * C < ((int64_t)1 << 40), "maxpool: shape");
  auto y = at::empty({N, C, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto code = at::empty({N, OH, OW, C}, x.options().dtype(at::kByte));
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  kfac::maxpool_nhwc_fwd(dtype_tag(x), x.data_ptr(), y.data_ptr(), code.data_ptr<uint8_t>(),
                         (int)N, (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p,
                         cur_stream());
  return {y, code};
}

at::Tensor maxpool_nhwc_bwd(const at::Tensor& gy, const at::Tensor& code, int64_t H, int64_t W,
                            int64_t k, int64_t s, int64_t p) {
  check_pool_input(gy, "maxpool gradient");
  const int64_t N = gy.size(0), C = gy.size(1), OH = gy.size(2), OW = gy.size(3);
  TORCH_CHECK(k >= 1 && k <= 15 && s >= 1 && p >= 0 && 2 * p <= k &&
                  OH == (H + 2 * p - k) / s + 1 && OW == (W + 2 * p - k) / s + 1,
              "maxpool_bwd: geometry");
  TORCH_CHECK(code.scalar_type() == at::kByte && code.is_contiguous() && code.dim() == 4 &&
                  code.size(0) == N && code.size(1) == OH && code.size(2) == OW &&
                  code.size(3) == C && code.device() == gy.device(),
              "maxpool_bwd: code must be the forward's uint8 [N, OH, OW, C]");
  auto gx = at::empty({N, C, H, W}, gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuardMasqueradingAsCUDA g(gy.device());
  kfac::maxpool_nhwc_bwd(dtype_tag(gy), gy.data_ptr(), code.data_ptr<uint8_t>(), gx.data_ptr(),
                         (int)N, (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p,
                         cur_stream());
  return gx;
}

void gemm3_grouped(const at::Tensor& table, int64_t nlayers, int64_t total_tiles,
                   bool a_kc, bool b_kc) {
  check_cuda(table, "table");
  TORCH_CHECK(table.numel() == nlayers * (int64_t)sizeof(kfac::GemmDesc),
              "gemm3: table size does not match the layer count");
  c10::hip::HIPGuardMasqueradingAsCUDA g(table.device());
  kfac::gemm3_grouped((const kfac::GemmDesc*)table.data_ptr(), (int)nlayers,
                      (int)total_tiles, a_kc, b_kc, cur_stream());
}

}  // namespace


// ------------------------------------------------------------ fused BN
namespace {
bool bn_ok(const at::Tensor& t) {
  return t.is_cuda() && (t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat) &&
         t.dim() == 4 &&
         t.is_contiguous(at::MemoryFormat::ChannelsLast) &&
         (reinterpret_cast<uintptr_t>(t.data_ptr()) % 16) == 0;
}
const float* opt_f(const c10::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr;
}
}  // namespace

bool bn_act_supported(const at::Tensor& x) {
  if (!bn_ok(x)) return false;
  const int64_t C = x.size(1);
  return C % 8 == 0 && C <= kfac::bn_max_c();
}

// x: [N, C, H, W] channels_last bf16.  Returns (y, stats[4, C] fp32).
std::vector<at::Tensor> bn_act_forward(const at::Tensor& x,
                                       const c10::optional<at::Tensor>& residual,
                                       const c10::optional<at::Tensor>& weight,
                                       const c10::optional<at::Tensor>& bias,
                                       const c10::optional<at::Tensor>& running_mean,
                                       const c10::optional<at::Tensor>& running_var,
                                       const c10::optional<at::Tensor>& num_batches,
                                       double momentum, double eps, bool relu,
                                       const c10::optional<at::Tensor>& ext_part) {
  TORCH_CHECK(bn_act_supported(x), "bn_act_forward: unsupported input");
  const int64_t C = x.size(1), M = x.numel() / C;
  const bool has_res = residual.has_value() && residual->defined();
  if (has_res) {
    TORCH_CHECK(bn_ok(*residual) && residual->sizes() == x.sizes() &&
                    residual->scalar_type() == x.scalar_type(),
                "residual layout");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  int64_t rpb;
  int nblk;
  kfac::bn_partition(M, (int)C, &rpb, &nblk);
  auto fopts = x.options().dtype(at::kFloat);
  auto part = at::empty({(int64_t)nblk * 2 * C}, fopts);
  auto stats = at::empty({4, C}, fopts);
  auto y = at::empty_like(x, at::MemoryFormat::ChannelsLast);
  int64_t* nb = nullptr;
  if (num_batches.has_value() && num_batches->defined()) {
    TORCH_CHECK(num_batches->scalar_type() == at::kLong && num_batches->is_cuda());
    nb = num_batches->data_ptr<int64_t>();
  }
  float* rm = running_mean.has_value() && running_mean->defined()
                  ? running_mean->data_ptr<float>() : nullptr;
  float* rv = running_var.has_value() && running_var->defined()
                  ? running_var->data_ptr<float>() : nullptr;
  // ext_part: the statistics partials of the convolution that produced x
  // ([P][2][C], GemmDesc::bnpart): no statistics pass over x
  const float* ep = nullptr;
  int ext_p = 0;
  if (ext_part.has_value() && ext_part->defined()) {
    check_cuda(*ext_part, "ext_part");
    TORCH_CHECK(x.scalar_type() == at::kFloat && ext_part->scalar_type() == at::kFloat &&
                    ext_part->is_contiguous() && ext_part->numel() % (2 * C) == 0 &&
                    ext_part->numel() / (2 * C) == 2 * ((M + 127) / 128),
                "bn_act_forward: ext_part must be the producer's fp32 [2 * ceil(M / 128)][2][C]");
    ep = ext_part->data_ptr<float>();
    ext_p = (int)(ext_part->numel() / (2 * C));
  }
  kfac::bn_forward(dtype_tag(x), x.data_ptr(), has_res ? residual->data_ptr() : nullptr,
                   opt_f(weight), opt_f(bias), rm, rv, nb, (float)momentum, (float)eps,
                   relu ? 1 : 0, M, (int)C, part.data_ptr<float>(), stats.data_ptr<float>(),
                   y.data_ptr(), cur_stream(), ep, ext_p);
  return {y, stats};
}

// Returns (dx, dweight, dbias, dresidual-or-undefined).
std::vector<at::Tensor> bn_act_backward(const at::Tensor& x, const at::Tensor& dy,
                                        const at::Tensor& y,
                                        const c10::optional<at::Tensor>& weight,
                                        const at::Tensor& stats, bool relu,
                                        bool has_res) {
  TORCH_CHECK(bn_act_supported(x) && stats.is_contiguous());
  const int64_t C = x.size(1), M = x.numel() / C;
  at::Tensor g = dy;
  if (!bn_ok(g) || g.scalar_type() != x.scalar_type())
    g = dy.to(x.scalar_type()).contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(bn_ok(y) && y.scalar_type() == x.scalar_type());
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  int64_t rpb;
  int nblk;
  kfac::bn_partition(M, (int)C, &rpb, &nblk);
  auto fopts = x.options().dtype(at::kFloat);
  auto part = at::empty({(int64_t)nblk * 2 * C}, fopts);
  auto coef = at::empty({3, C}, fopts);
  auto dw = at::empty({C}, fopts), db = at::empty({C}, fopts);
  auto dx = at::empty_like(x, at::MemoryFormat::ChannelsLast);
  at::Tensor dres;
  if (has_res) dres = at::empty_like(x, at::MemoryFormat::ChannelsLast);
  kfac::bn_backward(dtype_tag(x), x.data_ptr(), g.data_ptr(), y.data_ptr(), opt_f(weight),
                    stats.data_ptr<float>(), relu ? 1 : 0, M, (int)C,
                    part.data_ptr<float>(), coef.data_ptr<float>(), dw.data_ptr<float>(),
                    db.data_ptr<float>(), dx.data_ptr(), has_res ? dres.data_ptr() : nullptr,
                    cur_stream());
  return {dx, dw, db, dres};
}


// C++ autograd node for the fused BN: forward and backward never enter
// Python (a Python autograd.Function costs ~10-20 us of host time per call
// and per backward, ~2 ms per eager ResNet-50 step).
struct BNActFn : public torch::autograd::Function<BNActFn> {
  // every tensor argument must be defined (autograd records its device):
  // without a residual the caller passes x again and has_res = false
  static at::Tensor forward(torch::autograd::AutogradContext* ctx, const at::Tensor& x,
                            const at::Tensor& weight, const at::Tensor& bias,
                            const at::Tensor& residual, at::Tensor running_mean,
                            at::Tensor running_var, at::Tensor num_batches,
                            double momentum, double eps, bool relu, bool has_res,
                            const c10::optional<at::Tensor>& ext_part) {
    auto out = bn_act_forward(x, has_res ? c10::optional<at::Tensor>(residual) : c10::nullopt,
                              weight, bias, running_mean, running_var, num_batches,
                              momentum, eps, relu, ext_part);
    ctx->save_for_backward({x, out[0], weight, out[1]});
    ctx->saved_data["relu"] = relu;
    ctx->saved_data["has_res"] = has_res;
    return out[0];
  }
  static torch::autograd::variable_list backward(torch::autograd::AutogradContext* ctx,
                                                 torch::autograd::variable_list grads) {
    auto saved = ctx->get_saved_variables();
    const bool relu = ctx->saved_data["relu"].toBool();
    const bool has_res = ctx->saved_data["has_res"].toBool();
    auto r = bn_act_backward(saved[0], grads[0], saved[1], saved[2], saved[3], relu, has_res);
    at::Tensor undef;
    return {r[0], r[1], r[2], has_res ? r[3] : undef,
            undef, undef, undef, undef, undef, undef, undef, undef};
  }
};

// affine BN with running statistics (the Python side checks eligibility)
at::Tensor bn_act(const at::Tensor& x, const at::Tensor& weight, const at::Tensor& bias,
                  const c10::optional<at::Tensor>& residual,
                  const at::Tensor& running_mean, const at::Tensor& running_var,
                  const at::Tensor& num_batches, double momentum, double eps, bool relu,
                  const c10::optional<at::Tensor>& ext_part) {
  const bool has_res = residual.has_value() && residual->defined();
  return BNActFn::apply(x, weight, bias, has_res ? *residual : x, running_mean, running_var,
                        num_batches, momentum, eps, relu, has_res, ext_part);
}

// tridiag_host.cpp
std::vector<at::Tensor> tridiag_eigh_dc(const at::Tensor& d, const at::Tensor& e);
std::vector<int64_t> tridiag_dc_plan(int64_t n);
// twostage_host.cpp
std::vector<at::Tensor> eigh_twostage(const at::Tensor& A, bool timed);
int64_t eigh_twostage_max_n();

// ---- native batched fp32 GEMM (csrc/gemm_f32.hip) ----------------------
// 3-D fp32 CUDA views [batch, rows, cols] with unit column stride (any row /
// batch stride; a 2-D tensor is a batch of one).  C = alpha op(A) op(B) +
// beta C, op = transpose when ta / tb.
namespace {
struct Mat3 {
  int64_t b, r, c, ld, sb;
  float* p;
};
Mat3 mat3(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat, name, ": fp32 CUDA tensor");
  TORCH_CHECK(t.dim() == 2 || t.dim() == 3, name, ": 2-D or 3-D");
  const bool three = t.dim() == 3;
  Mat3 m{three ? t.size(0) : 1, t.size(three ? 1 : 0), t.size(three ? 2 : 1),
         t.stride(three ? 1 : 0), three ? t.stride(0) : 0, t.data_ptr<float>()};
  TORCH_CHECK(t.stride(three ? 2 : 1) == 1 || m.c == 1, name, ": unit column stride");
  if (m.r == 1) m.ld = std::max<int64_t>(m.ld, m.c);
  return m;
}
}  // namespace

void gemm_f32(const at::Tensor& a, const at::Tensor& b, at::Tensor& c, bool ta, bool tb,
              double alpha, double beta) {
  const Mat3 A = mat3(a, "a"), B = mat3(b, "b"), C = mat3(c, "c");
  const int64_t M = ta ? A.c : A.r, K = ta ? A.r : A.c;
  const int64_t Kb = tb ? B.c : B.r, N = tb ? B.r : B.c;
  TORCH_CHECK(K == Kb && C.r == M && C.c == N, "gemm_f32: shape mismatch");
  const int64_t batch = C.b;
  TORCH_CHECK((A.b == batch || A.b == 1) && (B.b == batch || B.b == 1),
              "gemm_f32: batch mismatch");
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31) && batch < 65536);
  c10::hip::HIPGuardMasqueradingAsCUDA g(c.device());
  gemm_native(ta, tb, (int)M, (int)N, (int)K, (float)alpha, A.p, A.ld,
                         A.b == 1 ? 0 : A.sb, B.p, B.ld, B.b == 1 ? 0 : B.sb, (float)beta, C.p,
                         C.ld, C.sb, (int)batch, cur_stream(), c.options());
}

// T <- T^-1 in place for a batch of upper-triangular [batch, n, n] fp32
void trinv_upper_(at::Tensor& t) {
  const Mat3 T = mat3(t, "t");
  TORCH_CHECK(T.r == T.c, "trinv_upper_: square matrices");
  c10::hip::HIPGuardMasqueradingAsCUDA g(t.device());
  auto work = at::empty({std::max<int64_t>(T.b * T.r * T.r / 2 + T.r, 1)}, t.options());
  kfac::trinv_upper_batched(T.p, T.ld, T.sb == 0 ? T.r * T.ld : T.sb, (int)T.r, (int)T.b,
                            work.data_ptr<float>(), cur_stream());
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X (gfx950) HIP kernels for distributed K-FAC";
  m.def("triu_pack", &triu_pack);
  m.def("triu_unpack", &triu_unpack);
  m.def("scale_copy", &scale_copy);
  m.def("syrk", &syrk, py::arg("x"), py::arg("C"), py::arg("bias"),
        py::arg("alpha"), py::arg("beta"), py::arg("splits") = 0,
        py::arg("alpha_scale") = py::none(), py::arg("fp32_exact") = false);
  m.def("syrk_default_splits", &kfac::syrk_workspace_splits);
  m.def("syrk_conv", &syrk_conv, py::arg("x"), py::arg("C"), py::arg("kh"), py::arg("kw"),
        py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("bias"),
        py::arg("alpha"), py::arg("beta"), py::arg("splits") = 0,
        py::arg("alpha_scale") = py::none(), py::arg("fp32_exact") = false);
  m.def("im2col", &im2col);
  m.def("eigen_scale", &eigen_scale);
  m.def("kl_dot", &kl_dot);
  m.def("kl_finalize", &kl_finalize);
  m.def("apply_grad", &apply_grad);
  m.def("fill_identity", &fill_identity);
  m.def("gemm_f32", &gemm_f32, py::arg("a"), py::arg("b"), py::arg("c"), py::arg("ta"),
        py::arg("tb"), py::arg("alpha") = 1.0, py::arg("beta") = 0.0);
  m.def("trinv_upper_", &trinv_upper_);
  m.def("jacobi_eigh", &jacobi_eigh);
  m.def("jacobi_max_n", &kfac::jacobi_max_n);
  m.def("build_layer_table", &build_layer_table, py::arg("ps"), py::arg("ws"),
        py::arg("bs"), py::arg("host") = py::none(),
        py::arg("bscales") = std::vector<double>());
  m.def("kl_dot_multi", &kl_dot_multi);
  m.def("kl_finalize_dev", &kl_finalize_dev);
  m.def("kl_reduce_partials", &kl_reduce_partials);
  m.def("apply_multi", &apply_multi);
  // GIL released: several host threads can each drive rocSOLVER on their
  // own stream (rocSOLVER's syevd blocks its calling thread internally)
  m.def("sytrd_nb", &sytrd_panel);
  m.def("sytrd_max_n", &sytrd_max_n);
  m.def("bn_act_supported", &bn_act_supported);
  m.def("bn_act_forward", &bn_act_forward, py::arg("x"), py::arg("residual"), py::arg("weight"),
        py::arg("bias"), py::arg("running_mean"), py::arg("running_var"),
        py::arg("num_batches"), py::arg("momentum"), py::arg("eps"), py::arg("relu"),
        py::arg("ext_part") = py::none());
  m.def("bn_act_backward", &bn_act_backward);
  m.def("bn_act", &bn_act, py::arg("x"), py::arg("weight"), py::arg("bias"), py::arg("residual"),
        py::arg("running_mean"), py::arg("running_var"), py::arg("num_batches"),
        py::arg("momentum"), py::arg("eps"), py::arg("relu"), py::arg("ext_part") = py::none());
  m.def("spd_inverse_blocked", &spd_inverse_blocked, py::call_guard<py::gil_scoped_release>());
  m.def("sytrd_reduce", &sytrd_reduce, py::call_guard<py::gil_scoped_release>());
  m.def("sytrd_begin", &sytrd_begin, py::call_guard<py::gil_scoped_release>());
  m.def("sytrd_advance", &sytrd_advance, py::arg("descs"), py::arg("sizes"), py::arg("k0"),
        py::arg("k1"), py::arg("waves") = 0, py::call_guard<py::gil_scoped_release>());
  m.def("rocsolver_eigh", &rocsolver_eigh, py::call_guard<py::gil_scoped_release>(),
        py::arg("A"), py::arg("algo") = 0,
        py::arg("max_sweeps") = 100, py::arg("tol") = 1e-7);
  m.def("build_gemm_table", &build_gemm_table, py::arg("As"), py::arg("A_extras"),
        py::arg("Bs"), py::arg("Cs"), py::arg("Ss"), py::arg("dgs"), py::arg("das"),
        py::arg("dampings"), py::arg("a_kc"), py::arg("b_kc"),
        py::arg("host") = py::none(),
        py::arg("A_hls") = std::vector<c10::optional<at::Tensor>>(),
        py::arg("B_hls") = std::vector<c10::optional<at::Tensor>>());
  m.def("gemm3_grouped", &gemm3_grouped);
  m.def("subsample_fwd", &subsample_fwd, py::arg("x"), py::arg("sh"), py::arg("sw"));
  m.def("sum_splits", &sum_splits, py::arg("part"), py::arg("out") = py::none());
  m.def("maxpool_nhwc_fwd", &maxpool_nhwc_fwd, py::arg("x"), py::arg("k"), py::arg("s"),
        py::arg("p"));
  m.def("maxpool_nhwc_bwd", &maxpool_nhwc_bwd, py::arg("gy"), py::arg("code"), py::arg("H"),
        py::arg("W"), py::arg("k"), py::arg("s"), py::arg("p"));
  m.def("col2im_nhwc", &col2im_nhwc, py::arg("cols"), py::arg("B"), py::arg("C"), py::arg("H"),
        py::arg("W"), py::arg("kh"), py::arg("kw"), py::arg("stride"), py::arg("pad"));
  m.def("pad_channels4", &pad_channels4, py::arg("x"));
  m.def("subsample_bwd_acc", &subsample_bwd_acc, py::arg("gy"), py::arg("gx"), py::arg("sh"),
        py::arg("sw"));
  m.def("subsample_bwd", &subsample_bwd, py::arg("gy"), py::arg("h"), py::arg("w"),
        py::arg("sh"), py::arg("sw"));
  m.def("gemm3_conv_wgrad", &gemm3_conv_wgrad, py::arg("x"), py::arg("dy"), py::arg("kh"),
        py::arg("kw"), py::arg("stride"), py::arg("pad"));
  m.def("gemm3_conv", &gemm3_conv, py::arg("x"), py::arg("w"), py::arg("stride"), py::arg("pad"),
        py::arg("flipw") = false, py::arg("bnpart") = py::none());
  m.def("gemm3_conv_splits",
        [](int64_t n, int64_t h, int64_t w, int64_t c, int64_t co, int64_t kh, int64_t kw,
           int64_t stride, int64_t pad) {
          return kfac::gemm3_conv_splits((int)n, (int)h, (int)w, (int)c, (int)co, (int)kh,
                                         (int)kw, (int)stride, (int)pad);
        });
  m.def("gemm3_mm", &gemm3_mm, py::arg("a"), py::arg("b"), py::arg("c"), py::arg("a_kc"),
        py::arg("b_kc"), py::arg("splits") = 1, py::arg("bnpart") = py::none(),
        py::arg("addend") = py::none());
  m.def("gemm3_mm_splits", &gemm3_mm_splits_for, py::arg("k"), py::arg("want"));
  m.def("gemm3s_align", &kfac::gemm3s_align);
  m.def("build_gemm3s_table", &build_gemm3s_table);
  m.def("gemm3s_grouped", &gemm3s_grouped);
  m.def("build_split_table", &build_split_table);
  m.def("split_pad_multi", &split_pad_multi);
  m.def("build_cast_table", &build_cast_table);
  m.def("cast_multi", &cast_multi);
  // GIL released: one host thread per eigensolver lane (the sweep loop reads
  // its convergence flags back once per sweep)
  m.def("tridiag_eigh_dc", &tridiag_eigh_dc, py::call_guard<py::gil_scoped_release>());
  m.def("tridiag_dc_plan", &tridiag_dc_plan);
  m.def("eigh_twostage", &eigh_twostage, py::call_guard<py::gil_scoped_release>(),
        py::arg("A"), py::arg("timed") = false);
  m.def("eigh_twostage_max_n", &eigh_twostage_max_n);
  m.def("flush_table_uploads", &flush_table_uploads);
  m.def("register_table_slot", &register_table_slot);
  m.def("memset_raw", &memset_raw);
  m.def("unregister_table_slot", &unregister_table_slot);
  m.attr("arch") = "gfx950";
}
