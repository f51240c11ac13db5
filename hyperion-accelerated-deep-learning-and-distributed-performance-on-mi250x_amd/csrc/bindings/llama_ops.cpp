// Torch bindings: rotary embeddings and SwiGLU (Llama elementwise kernels).
#include "bindings/common.h"
#include "bindings/registry.h"

namespace hypbind {
namespace {

void check_rope_operand(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4, name, ": expected a [B, S, H, D] GPU tensor");
  TORCH_CHECK(t.stride(3) == 1, name, ": head dim must be contiguous");
  TORCH_CHECK(t.stride(0) == t.size(1) * t.stride(1), name, ": batch and sequence dims must be mergeable");
  TORCH_CHECK(t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              name, ": strides / base must be 16-byte aligned");
}

// q [B,S,Hq,D], k [B,S,Hk,D] -> rotated copies (contiguous); positions int64 [B,S] or None
std::vector<at::Tensor> rope(const at::Tensor& q, const at::Tensor& k, const c10::optional<at::Tensor>& positions,
                             double theta, bool inverse) {
  check_rope_operand(q, "rope q");
  check_rope_operand(k, "rope k");
  TORCH_CHECK(q.size(0) == k.size(0) && q.size(1) == k.size(1) && q.size(3) == k.size(3), "rope: q/k shape mismatch");
  TORCH_CHECK(q.scalar_type() == k.scalar_type(), "rope: q/k dtype mismatch");
  const int64_t D = q.size(3);
  TORCH_CHECK(D % 16 == 0, "rope: head_dim must be a multiple of 16");
  const int64_t* pos = nullptr;
  at::Tensor pc;
  if (positions.has_value() && positions->defined()) {
    pc = positions->to(at::kLong).contiguous();
    TORCH_CHECK(pc.numel() == q.size(0) * q.size(1), "rope: positions must be [B, S]");
    pos = pc.data_ptr<int64_t>();
  }
  const at::DeviceGuard guard(q.device());
  auto qo = at::empty(q.sizes(), q.options());
  auto ko = at::empty(k.sizes(), k.options());
  // outputs are contiguous: token stride H*D, head stride D; inputs keep their own strides, so
  // the kernel reads through in-strides and writes out-strides -> use the contiguous layout for both
  // by passing input strides (outputs share them only if inputs are contiguous)
  at::Tensor qi = q, ki = k;
  if (q.stride(1) != q.size(2) * D || q.stride(2) != D) qi = q.contiguous();
  if (k.stride(1) != k.size(2) * D || k.stride(2) != D) ki = k.contiguous();
  HYP_CHECK_HIP(hyp::rope_apply(dtype_code(q), qi.data_ptr(), ki.data_ptr(), qo.data_ptr(), ko.data_ptr(),
                                q.size(0) * q.size(1), (int)q.size(1), (int)q.size(2), (int)k.size(2), (int)D,
                                q.size(2) * D, k.size(2) * D, D, D, pos, (float)theta, inverse ? 1 : 0, cur_stream()));
  return {qo, ko};
}

// in place on strided [B, S, H, D] views (e.g. the q / k columns of a packed [B*S, 3*H*D] buffer):
// the kernel reads each lane's pairs before writing them back
void rope_inplace(at::Tensor& q, at::Tensor& k, const c10::optional<at::Tensor>& positions, double theta,
                  bool inverse) {
  check_rope_operand(q, "rope_ q");
  check_rope_operand(k, "rope_ k");
  TORCH_CHECK(q.sizes() == k.sizes() && q.scalar_type() == k.scalar_type(), "rope_: q/k mismatch");
  const int64_t D = q.size(3);
  TORCH_CHECK(D % 16 == 0, "rope_: head_dim must be a multiple of 16");
  const int64_t* pos = nullptr;
  at::Tensor pc;
  if (positions.has_value() && positions->defined()) {
    pc = positions->to(at::kLong).contiguous();
    TORCH_CHECK(pc.numel() == q.size(0) * q.size(1), "rope_: positions must be [B, S]");
    pos = pc.data_ptr<int64_t>();
  }
  const at::DeviceGuard guard(q.device());
  HYP_CHECK_HIP(hyp::rope_apply(dtype_code(q), q.data_ptr(), k.data_ptr(), q.data_ptr(), k.data_ptr(),
                                q.size(0) * q.size(1), (int)q.size(1), (int)q.size(2), (int)k.size(2), (int)D,
                                q.stride(1), k.stride(1), q.stride(2), k.stride(2), pos, (float)theta, inverse ? 1 : 0,
                                cur_stream()));
}

at::Tensor swiglu_fwd(const at::Tensor& g, const at::Tensor& u) {
  TORCH_CHECK(g.is_cuda() && g.sizes() == u.sizes() && g.scalar_type() == u.scalar_type(), "swiglu: g/u mismatch");
  TORCH_CHECK(g.numel() % 8 == 0, "swiglu: numel must be a multiple of 8");
  const at::DeviceGuard guard(g.device());
  auto gc = g.contiguous(), uc = u.contiguous();
  auto h = at::empty_like(gc);
  HYP_CHECK_HIP(hyp::swiglu_forward(dtype_code(g), gc.data_ptr(), uc.data_ptr(), h.data_ptr(), g.numel(), cur_stream()));
  return h;
}

std::vector<at::Tensor> swiglu_bwd(const at::Tensor& dh, const at::Tensor& g, const at::Tensor& u) {
  TORCH_CHECK(dh.sizes() == g.sizes() && g.sizes() == u.sizes(), "swiglu_bwd: shape mismatch");
  TORCH_CHECK(dh.scalar_type() == g.scalar_type() && g.scalar_type() == u.scalar_type(), "swiglu_bwd: dtype mismatch");
  const at::DeviceGuard guard(g.device());
  auto dhc = dh.contiguous(), gc = g.contiguous(), uc = u.contiguous();
  auto dg = at::empty_like(gc), du = at::empty_like(uc);
  HYP_CHECK_HIP(hyp::swiglu_backward(dtype_code(g), dhc.data_ptr(), gc.data_ptr(), uc.data_ptr(), dg.data_ptr(),
                                     du.data_ptr(), g.numel(), cur_stream()));
  return {dg, du};
}

}  // namespace

void register_llama_ops(pybind11::module& m) {
  m.def("rope", &rope, "rotary position embedding on q and k (HF rotate_half convention)");
  m.def("rope_", &rope_inplace, "in-place rotary embedding on strided q / k views");
  m.def("swiglu_fwd", &swiglu_fwd, "silu(g) * u");
  m.def("swiglu_bwd", &swiglu_bwd, "SwiGLU backward -> (dg, du)");
}

}  // namespace hypbind
