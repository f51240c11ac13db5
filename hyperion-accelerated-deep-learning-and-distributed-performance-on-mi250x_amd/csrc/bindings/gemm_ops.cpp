// Torch bindings: hand-written MFMA GEMM (microbenchmarks + building block).
#include "bindings/common.h"
#include "bindings/registry.h"

namespace hypbind {
namespace {

// a [M, K], b [N, K] (both K-contiguous) -> a @ b.T in out_dtype ("" = same as inputs)
at::Tensor gemm_nt(const at::Tensor& a, const at::Tensor& b, c10::optional<at::ScalarType> out_dtype, double alpha,
                   int64_t bk) {
  HYP_CHECK_CUDA_TENSOR(a);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(1), "gemm_nt: expected a [M,K], b [N,K]");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1, "gemm_nt: K must be contiguous");
  TORCH_CHECK(a.scalar_type() == b.scalar_type() && (a.scalar_type() == at::kBFloat16 || a.scalar_type() == at::kHalf),
              "gemm_nt: bf16/f16 inputs of one dtype");
  const int M = (int)a.size(0), N = (int)b.size(0), K = (int)a.size(1);
  TORCH_CHECK(hyp::gemm_nt_supported(M, N, K, (int)a.stride(0), (int)b.stride(0), (int)bk),
              "gemm_nt: shape not supported (M, N multiples of 128; K multiple of bk; 16-byte rows)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0,
              "gemm_nt: 16-byte aligned bases required");
  const at::DeviceGuard guard(a.device());
  auto c = at::empty({M, N}, a.options().dtype(out_dtype.has_value() ? *out_dtype : a.scalar_type()));
  HYP_CHECK_HIP(hyp::gemm_nt(dtype_code(a), dtype_code(c), a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K,
                             (int)a.stride(0), (int)b.stride(0), N, (float)alpha, (int)bk, cur_stream()));
  return c;
}

}  // namespace

void register_gemm_ops(pybind11::module& m) {
  m.def("gemm_nt", &gemm_nt, "C = alpha * A @ B.T on MFMA (bf16/f16 in)", pybind11::arg("a"), pybind11::arg("b"),
        pybind11::arg("out_dtype") = pybind11::none(), pybind11::arg("alpha") = 1.0, pybind11::arg("bk") = 64);
}

}  // namespace hypbind
