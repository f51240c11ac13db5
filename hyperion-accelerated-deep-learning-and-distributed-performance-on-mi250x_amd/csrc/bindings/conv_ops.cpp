// Torch bindings: implicit-GEMM convolution (+ BN-statistics epilogue) and BN from partials.
#include "bindings/common.h"
#include "bindings/registry.h"

namespace hypbind {
namespace {

at::Tensor& zero_page(const at::Device& dev) {
  static at::Tensor z[16];
  const int i = dev.index() < 0 ? 0 : dev.index();
  if (!z[i].defined()) z[i] = at::zeros({4096}, at::TensorOptions().device(dev).dtype(at::kByte));
  return z[i];
}

// x [N,C,H,W] channels-last, w [K,C,R,S] channels-last -> (y [N,K,P,Q] channels-last, psum, psq)
std::vector<at::Tensor> conv_fwd(const at::Tensor& x, const at::Tensor& w, int64_t sh, int64_t sw, int64_t ph,
                                 int64_t pw, bool stats) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4, "conv_fwd: 4D tensors");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) && w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_fwd: channels-last input and weight required");
  TORCH_CHECK(x.scalar_type() == w.scalar_type() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf),
              "conv_fwd: bf16/f16 input and weight of one dtype");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int K = w.size(0), R = w.size(2), S = w.size(3);
  TORCH_CHECK(w.size(1) == C, "conv_fwd: channel mismatch");
  TORCH_CHECK(hyp::conv_fwd_supported(C, K), "conv_fwd: needs C % 64 == 0 and K % 8 == 0");
  const int P = (H + 2 * ph - R) / sh + 1, Q = (W + 2 * pw - S) / sw + 1;
  TORCH_CHECK(P > 0 && Q > 0, "conv_fwd: empty output");
  const at::DeviceGuard guard(x.device());
  auto y = at::empty({N, K, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int M = N * P * Q;
  int bm = 128, bn = 128;
  hyp::conv_fwd_tile(M, K, &bm, &bn);
  at::Tensor psum, psq;
  if (stats) {
    const int mt = (M + bm - 1) / bm;
    auto part = at::empty({2, mt, K}, x.options().dtype(at::kFloat));
    psum = part[0];
    psq = part[1];
  }
  HYP_CHECK_HIP(hyp::conv_fwd(dtype_code(x), x.data_ptr(), w.data_ptr(), y.data_ptr(), zero_page(x.device()).data_ptr(),
                              stats ? psum.data_ptr<float>() : nullptr, stats ? psq.data_ptr<float>() : nullptr, N, H, W,
                              C, K, P, Q, R, S, (int)sh, (int)sw, (int)ph, (int)pw, bm, bn, cur_stream()));
  return {y, psum, psq};
}

// BN forward (training) given conv-epilogue partials: returns (y, save_mean, save_invstd)
std::vector<at::Tensor> bn_fwd_partials(const at::Tensor& x, const c10::optional<at::Tensor>& residual,
                                        const at::Tensor& psum, const at::Tensor& psq,
                                        const c10::optional<at::Tensor>& weight, const c10::optional<at::Tensor>& bias,
                                        const c10::optional<at::Tensor>& running_mean,
                                        const c10::optional<at::Tensor>& running_var, double momentum, double eps,
                                        bool act) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(is_rows_by_channels(x), "bn_fwd_partials: x must be channels-last");
  const int64_t C = x.size(1), M = x.numel() / C;
  TORCH_CHECK(psum.dim() == 2 && psum.size(1) == C && psq.sizes() == psum.sizes(), "bn_fwd_partials: partials shape");
  if (residual.has_value() && residual->defined())
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->scalar_type() == x.scalar_type() &&
                    is_rows_by_channels(*residual),
                "bn_fwd_partials: residual shape/dtype/layout mismatch");
  const at::DeviceGuard guard(x.device());
  auto y = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto stats = at::empty({2, C}, fopt);
  auto ws = at::empty({2 * C}, fopt);
  HYP_CHECK_HIP(hyp::bn_forward_from_partials(
      dtype_code(x), x.data_ptr(), vptr_or_null(residual), y.data_ptr(), M, (int)C, ptr_or_null<float>(weight),
      ptr_or_null<float>(bias), ptr_or_null<float>(running_mean), ptr_or_null<float>(running_var), (float)momentum,
      (float)eps, act ? 1 : 0, psum.data_ptr<float>(), psq.data_ptr<float>(), (int)psum.size(0), stats.data_ptr<float>(),
      stats.data_ptr<float>() + C, ws.data_ptr<float>(), ws.data_ptr<float>() + C, cur_stream()));
  return {y, stats[0], stats[1]};
}

}  // namespace

void register_conv_ops(pybind11::module& m) {
  m.def("conv_fwd", &conv_fwd, "NHWC implicit-GEMM conv on MFMA (+ BN statistics partials)");
  m.def("bn_fwd_partials", &bn_fwd_partials, "BN finalize + apply from conv-epilogue partials");
}

}  // namespace hypbind
