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

// fp32 a [M, K], b [N, K] -> a @ b.T on the fp32-input MFMA (gemm_f32.hip)
at::Tensor gemm_f32_nt(const at::Tensor& a, const at::Tensor& b, c10::optional<at::ScalarType> out_dtype, double alpha) {
  HYP_CHECK_CUDA_TENSOR(a);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(1), "gemm_f32_nt: expected a [M,K], b [N,K]");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1, "gemm_f32_nt: K must be contiguous");
  TORCH_CHECK(a.scalar_type() == at::kFloat && b.scalar_type() == at::kFloat, "gemm_f32_nt: fp32 inputs");
  const int M = (int)a.size(0), N = (int)b.size(0), K = (int)a.size(1);
  TORCH_CHECK(hyp::gemm_f32_nt_supported(M, N, K, (int)a.stride(0), (int)b.stride(0)),
              "gemm_f32_nt: shape not supported (M, N multiples of 128; K multiple of 32; 16-byte rows)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0,
              "gemm_f32_nt: 16-byte aligned bases required");
  const at::DeviceGuard guard(a.device());
  auto c = at::empty({M, N}, a.options().dtype(out_dtype.has_value() ? *out_dtype : at::kFloat));
  HYP_CHECK_HIP(hyp::gemm_f32_nt(dtype_code(c), a.data_ptr<float>(), b.data_ptr<float>(), c.data_ptr(), M, N, K,
                                 (int)a.stride(0), (int)b.stride(0), N, (float)alpha, cur_stream()));
  return c;
}

// Operand view: a 2D tensor with unit stride in its last dim.  row form (tr = false): X[i, k] at
// row i; tr form: X is [K, I] with X(i, k) = X[k, i].
void check_operand(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.stride(0) % 8 == 0 && t.stride(0) >= t.size(1),
              "gemm: ", name, " must be 2D, unit stride in dim 1, row stride a multiple of 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "gemm: ", name, " base must be 16-byte aligned");
}

// C = epi(alpha · A·Bᵀ) with A [M, K] (a_tr: [K, M]) and B [N, K] (b_tr: [K, N]).
at::Tensor gemm(const at::Tensor& a, const at::Tensor& b, bool a_tr, bool b_tr, c10::optional<at::ScalarType> out_dtype,
                const c10::optional<at::Tensor>& bias, int64_t act, const c10::optional<at::Tensor>& aux,
                const c10::optional<at::Tensor>& residual, double alpha, double beta,
                const c10::optional<at::Tensor>& out, int64_t tile, int64_t splits, double drop_p,
                const c10::optional<at::Tensor>& rng, int64_t n_out) {
  HYP_CHECK_CUDA_TENSOR(a);
  check_operand(a, "a");
  check_operand(b, "b");
  TORCH_CHECK(a.scalar_type() == b.scalar_type() && (a.scalar_type() == at::kBFloat16 || a.scalar_type() == at::kHalf),
              "gemm: bf16/f16 operands of one dtype");
  const int64_t M = a_tr ? a.size(1) : a.size(0), K = a_tr ? a.size(0) : a.size(1);
  const int64_t NB = b_tr ? b.size(1) : b.size(0), Kb = b_tr ? b.size(0) : b.size(1);
  // n_out > rows of a row-form B: output columns past B's rows are computed from zeros (the LM
  // head's padded class columns, written so the padded logits buffer needs no separate fill)
  TORCH_CHECK(n_out < 0 || (!b_tr && n_out >= NB), "gemm: n_out needs a row-form b with at most n_out rows");
  const int64_t N = n_out > 0 ? n_out : NB;
  TORCH_CHECK(K == Kb, "gemm: reduction sizes differ (", K, " vs ", Kb, ")");
  TORCH_CHECK(N % 4 == 0 && (K % 8 == 0 || a_tr || b_tr) && (!a_tr || M % 8 == 0) && (!b_tr || N % 8 == 0),
              "gemm: needs N % 4 == 0, K % 8 == 0 unless an operand is transposed (and M / N % 8 == 0 for "
              "transposed operands)");
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31), "gemm: dims must fit int32");
  const at::DeviceGuard guard(a.device());
  at::Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    TORCH_CHECK(c.dim() == 2 && c.size(0) == M && c.size(1) == N && c.stride(1) == 1 && c.stride(0) % 4 == 0,
                "gemm: out must be [M, N] with unit column stride");
    TORCH_CHECK(!out_dtype.has_value() || *out_dtype == c.scalar_type(), "gemm: out dtype mismatch");
  } else {
    TORCH_CHECK(beta == 0.0, "gemm: beta needs out");
    c = at::empty({M, N}, a.options().dtype(out_dtype.has_value() ? *out_dtype : a.scalar_type()));
  }
  hyp::GemmTiledArgs g;
  g.in_dtype = dtype_code(a);
  g.out_dtype = dtype_code(c);
  g.A = a.data_ptr();
  g.B = b.data_ptr();
  g.C = c.data_ptr();
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  g.lda = (int)a.stride(0);
  g.ldb = (int)b.stride(0);
  g.ldc = (int)c.stride(0);
  g.a_tr = a_tr;
  g.b_tr = b_tr;
  g.act = (int)act;
  TORCH_CHECK(act >= 0 && act <= 3, "gemm: act is 0 (none), 1 (relu), 2 (gelu), 3 (gelu tanh)");
  g.alpha = (float)alpha;
  g.beta = (float)beta;
  g.tile = (int)tile;
  g.splits = (int)splits;
  g.b_rows = (int)NB;
  g.zero = device_zero_page(a.device());
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->dim() == 1 && bias->numel() == N && bias->is_contiguous(), "gemm: bias must be [N] contiguous");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(bias->data_ptr()) % 16 == 0, "gemm: bias must be 16-byte aligned");
    g.bias = bias->data_ptr();
    g.bias_dtype = dtype_code(*bias);
  }
  if (aux.has_value() && aux->defined()) {
    TORCH_CHECK(act != 0 && aux->sizes() == c.sizes() && aux->strides() == c.strides() &&
                    aux->scalar_type() == c.scalar_type(),
                "gemm: aux (pre-activation) must match out and needs an activation");
    g.aux = aux->data_ptr();
  }
  if (residual.has_value() && residual->defined()) {
    const at::Tensor& r = *residual;
    TORCH_CHECK(r.dim() == 2 && r.size(0) == M && r.size(1) == N && r.stride(1) == 1 && r.stride(0) % 4 == 0 &&
                    r.scalar_type() == c.scalar_type(),
                "gemm: residual must be [M, N], unit column stride, output dtype");
    g.R = r.data_ptr();
    g.ldr = (int)r.stride(0);
  }
  if (drop_p > 0.0) {  // dropout(act(...)) in the epilogue (the FFN's inner dropout)
    TORCH_CHECK(act != 0 && drop_p < 1.0 && rng.has_value() && rng->defined() && !g.R && c.stride(0) == N,
                "gemm: dropout needs an activation, p < 1, an rng record, no residual and a dense output");
    g.drop_p = (float)drop_p;
    g.drng = unpack_rng(*rng);
  }
  const int sp = hyp::gemm_tiled_splits(g);
  at::Tensor part;
  if (sp > 1) {
    part = at::empty({(int64_t)sp * M * N}, a.options().dtype(at::kFloat));
    g.part = part.data_ptr<float>();
  }
  HYP_CHECK_HIP(hyp::gemm_tiled(g, cur_stream()));
  return c;
}

std::vector<int64_t> gemm_plan(int64_t M, int64_t N, int64_t K) {
  int t, s;
  hyp::gemm_tiled_plan((int)M, (int)N, (int)K, &t, &s);
  return {t, s};
}

}  // namespace

void register_gemm_ops(pybind11::module& m) {
  m.def("gemm", &gemm, "C = epi(alpha A·Bᵀ): deep-pipelined MFMA GEMM, NT/NN/TN layouts, fused epilogue",
        pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("a_tr") = false, pybind11::arg("b_tr") = false,
        pybind11::arg("out_dtype") = pybind11::none(), pybind11::arg("bias") = pybind11::none(),
        pybind11::arg("act") = 0, pybind11::arg("aux") = pybind11::none(), pybind11::arg("residual") = pybind11::none(),
        pybind11::arg("alpha") = 1.0, pybind11::arg("beta") = 0.0, pybind11::arg("out") = pybind11::none(),
        pybind11::arg("tile") = -1, pybind11::arg("splits") = -1, pybind11::arg("drop_p") = 0.0,
        pybind11::arg("rng") = pybind11::none(), pybind11::arg("n_out") = -1);
  m.def("gemm_set_splitk_inkernel", [](int64_t on) { hyp::gemm_set_splitk_inkernel((int)on); },
        "A/B: split-K reduce in the last-arriving workgroup (1) or the separate reduce kernel (0, default)");
  m.def("gemm_plan", &gemm_plan, "(tile, splits) the automatic plan picks for an M x N x K GEMM");
  m.def("gemm_f32_nt", &gemm_f32_nt, "C = alpha * A @ B.T, fp32 in, on the fp32-input MFMA", pybind11::arg("a"),
        pybind11::arg("b"), pybind11::arg("out_dtype") = pybind11::none(), pybind11::arg("alpha") = 1.0);
  m.def("gemm_nt", &gemm_nt, "C = alpha * A @ B.T on MFMA (bf16/f16 in)", pybind11::arg("a"), pybind11::arg("b"),
        pybind11::arg("out_dtype") = pybind11::none(), pybind11::arg("alpha") = 1.0, pybind11::arg("bk") = 64);
}

}  // namespace hypbind
