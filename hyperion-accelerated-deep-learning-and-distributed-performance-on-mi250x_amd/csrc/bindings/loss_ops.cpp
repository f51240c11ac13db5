// Torch bindings: fused softmax cross-entropy (forward + in-place backward).
#include "bindings/common.h"
#include "bindings/registry.h"

namespace hypbind {
namespace {

// logits [N, V] (row stride ld >= V, unit column stride) is overwritten with dlogits when
// write_grad.  Returns (loss_rows [N] fp32, lse [N] fp32).
std::vector<at::Tensor> ce_fwd_bwd(at::Tensor& logits, const at::Tensor& target, const c10::optional<at::Tensor>& scale,
                                   double scale_mul, int64_t ignore_index, bool write_grad,
                                   const c10::optional<at::Tensor>& bias) {
  HYP_CHECK_CUDA_TENSOR(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "ce_fwd_bwd: logits must be [N, V] with unit column stride");
  TORCH_CHECK(target.dim() == 1 && target.size(0) == logits.size(0) && target.scalar_type() == at::kLong &&
                  target.is_contiguous() && target.device() == logits.device(),
              "ce_fwd_bwd: target must be a contiguous int64 [N] on the logits device");
  if (scale.has_value() && scale->defined())
    TORCH_CHECK(scale->scalar_type() == at::kFloat && scale->numel() == 1 && scale->device() == logits.device(),
                "ce_fwd_bwd: scale must be a 1-element fp32 device tensor");
  TORCH_CHECK(logits.size(1) < (int64_t)INT32_MAX, "ce_fwd_bwd: V too large");
  if (bias.has_value() && bias->defined())
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() == logits.size(1) &&
                    bias->device() == logits.device() && reinterpret_cast<uintptr_t>(bias->data_ptr()) % 16 == 0,
                "ce_fwd_bwd: bias must be a contiguous, 16-byte aligned fp32 [V] on the logits device");
  const at::DeviceGuard guard(logits.device());
  auto fopt = logits.options().dtype(at::kFloat);
  auto loss = at::empty({logits.size(0)}, fopt);
  auto lse = at::empty({logits.size(0)}, fopt);
  HYP_CHECK_HIP(hyp::cross_entropy_fwd_bwd(dtype_code(logits), logits.data_ptr(), logits.size(0), (int)logits.size(1),
                                           logits.stride(0), target.data_ptr<int64_t>(), loss.data_ptr<float>(),
                                           lse.data_ptr<float>(), ptr_or_null<float>(scale), (float)scale_mul,
                                           ignore_index, write_grad ? 1 : 0, cur_stream(), ptr_or_null<float>(bias)));
  return {loss, lse};
}

// ---- embedding ---------------------------------------------------------------------------------
at::Tensor embedding_fwd(const at::Tensor& ids, const at::Tensor& w) {
  HYP_CHECK_CUDA_TENSOR(w);
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous() && ids.device() == w.device(),
              "embedding_fwd: contiguous int64 ids on the weight's device");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && w.size(1) % 8 == 0, "embedding_fwd: contiguous [V, E], E % 8 == 0");
  const at::DeviceGuard guard(w.device());
  std::vector<int64_t> shape(ids.sizes().begin(), ids.sizes().end());
  shape.push_back(w.size(1));
  auto out = at::empty(shape, w.options());
  HYP_CHECK_HIP(hyp::embedding_forward(dtype_code(w), ids.data_ptr<int64_t>(), w.data_ptr(), out.data_ptr(),
                                       ids.numel(), (int)w.size(1), w.size(0), cur_stream()));
  return out;
}

// dy [..., E] (contiguous), ids [...] -> dense dW [V, E] (rows of absent ids and of pad_idx are zero)
at::Tensor embedding_bwd(const at::Tensor& dy, const at::Tensor& ids, int64_t V, int64_t pad_idx) {
  HYP_CHECK_CUDA_TENSOR(dy);
  const int64_t E = dy.size(-1), n = ids.numel();
  TORCH_CHECK(dy.is_contiguous() && dy.numel() == n * E && E % 8 == 0, "embedding_bwd: contiguous dy [..., E]");
  TORCH_CHECK(ids.is_contiguous() && ids.scalar_type() == at::kLong, "embedding_bwd: contiguous int64 ids");
  const at::DeviceGuard guard(dy.device());
  // fp32: the zeroed accumulator is the gradient; bf16 / f16: only the ids' rows are used (cleared
  // in-kernel), the rest of the scratch accumulator is never touched
  auto dw32 = dy.scalar_type() == at::kFloat ? at::zeros({V, E}, dy.options())
                                             : at::empty({V, E}, dy.options().dtype(at::kFloat));
  at::Tensor dw = dy.scalar_type() == at::kFloat ? dw32 : at::empty({V, E}, dy.options());
  HYP_CHECK_HIP(hyp::embedding_backward(dtype_code(dy), ids.data_ptr<int64_t>(), dy.data_ptr(),
                                        dw32.data_ptr<float>(), dw.data_ptr(), n, (int)E, V, pad_idx, cur_stream()));
  return dw;
}

}  // namespace

void register_loss_ops(pybind11::module& m) {
  m.def("embedding_fwd", &embedding_fwd, "token embedding gather");
  m.def("embedding_bwd", &embedding_bwd, "dense embedding gradient (fp32 atomic accumulate + cast)");
  m.def("ce_fwd_bwd", &ce_fwd_bwd, "in-place softmax cross-entropy forward+backward", pybind11::arg("logits"),
        pybind11::arg("target"), pybind11::arg("scale"), pybind11::arg("scale_mul"), pybind11::arg("ignore_index"),
        pybind11::arg("write_grad"), pybind11::arg("bias") = pybind11::none());
}

}  // namespace hypbind
