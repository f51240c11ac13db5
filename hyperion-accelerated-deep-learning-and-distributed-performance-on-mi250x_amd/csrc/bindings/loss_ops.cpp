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

// ---- classifier head + MSE (linear_mse.hip) -----------------------------------------------------
void check_head(const at::Tensor& x, const at::Tensor& w, const char* who) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.is_contiguous() && w.is_contiguous() && x.size(1) == w.size(1) &&
                  x.scalar_type() == w.scalar_type() && w.device() == x.device() && x.size(0) >= 1 &&
                  x.size(0) <= 64 && x.size(1) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              who, ": contiguous 16-byte aligned x [M <= 64, K % 8 == 0] and w [N, K] of one dtype and device");
}

// (loss fp32 scalar, dz fp32 [M, N])
std::vector<at::Tensor> linear_mse_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b,
                                       const at::Tensor& y) {
  check_head(x, w, "linear_mse_fwd");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(y.scalar_type() == at::kFloat && y.is_contiguous() && y.dim() == 2 && y.size(0) == M && y.size(1) == N &&
                  y.device() == x.device(), "linear_mse_fwd: y must be a contiguous fp32 [M, N]");
  if (b.has_value() && b->defined())
    TORCH_CHECK(b->scalar_type() == x.scalar_type() && b->is_contiguous() && b->numel() == N && b->device() == x.device(),
                "linear_mse_fwd: bias must be a contiguous [N] of x's dtype");
  const at::DeviceGuard guard(x.device());
  auto fopt = x.options().dtype(at::kFloat);
  auto loss = at::empty({}, fopt);
  auto dz = at::empty({M, N}, fopt);
  auto ws = at::empty({hyp::linear_mse_workspace((int)M, (int)N, (int)K)}, fopt);
  HYP_CHECK_HIP(hyp::linear_mse_fwd(dtype_code(x), x.data_ptr(), w.data_ptr(), vptr_or_null(b), y.data_ptr<float>(),
                                    (int)M, (int)N, (int)K, dz.data_ptr<float>(), ws.data_ptr<float>(),
                                    loss.data_ptr<float>(), cur_stream()));
  return {loss, dz};
}

// (dx [M, K], dw [N, K], db [N] or undefined) scaled by the fp32 device scalar go
std::vector<at::Tensor> linear_mse_bwd(const at::Tensor& dz, const at::Tensor& go, const at::Tensor& x,
                                       const at::Tensor& w, bool with_bias) {
  check_head(x, w, "linear_mse_bwd");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(dz.scalar_type() == at::kFloat && dz.is_contiguous() && dz.numel() == M * N && go.numel() == 1 &&
                  go.scalar_type() == at::kFloat && go.device() == x.device() && dz.device() == x.device(),
              "linear_mse_bwd: fp32 dz [M, N] and a 1-element fp32 go");
  const at::DeviceGuard guard(x.device());
  auto goc = go.contiguous();
  auto ws = at::empty({hyp::linear_mse_workspace((int)M, (int)N, (int)K)}, x.options().dtype(at::kFloat));
  auto dx = at::empty_like(x);
  auto dw = at::empty_like(w);
  at::Tensor db;
  if (with_bias) db = at::empty({N}, w.options());
  HYP_CHECK_HIP(hyp::linear_mse_bwd(dtype_code(x), dz.data_ptr<float>(), goc.data_ptr<float>(), x.data_ptr(),
                                    w.data_ptr(), (int)M, (int)N, (int)K, dx.data_ptr(), dw.data_ptr(),
                                    with_bias ? db.data_ptr() : nullptr, ws.data_ptr<float>(), cur_stream()));
  return {dx, dw, db};
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
  m.def("linear_mse_fwd", &linear_mse_fwd, "classifier head + MSE forward (loss, fp32 dz)", pybind11::arg("x"),
        pybind11::arg("w"), pybind11::arg("b"), pybind11::arg("y"));
  m.def("linear_mse_bwd", &linear_mse_bwd, "classifier head + MSE backward (dx, dw, db) in one launch",
        pybind11::arg("dz"), pybind11::arg("go"), pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("with_bias"));
  m.def("embedding_bwd", &embedding_bwd, "dense embedding gradient (fp32 atomic accumulate + cast)");
  m.def("ce_fwd_bwd", &ce_fwd_bwd, "in-place softmax cross-entropy forward+backward", pybind11::arg("logits"),
        pybind11::arg("target"), pybind11::arg("scale"), pybind11::arg("scale_mul"), pybind11::arg("ignore_index"),
        pybind11::arg("write_grad"), pybind11::arg("bias") = pybind11::none());
}

}  // namespace hypbind
