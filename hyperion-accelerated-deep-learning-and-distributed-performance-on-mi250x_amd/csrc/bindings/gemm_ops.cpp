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

// ---- fp32 (gemm_f32.hip) ---------------------------------------------------------------------
// C = epi(alpha · A·Bᵀ) in fp32, A [M, K] (a_tr: [K, M]), B [N, K] (b_tr: [K, N]); + beta·out, + bias,
// ReLU.  Any M / N; row-form operands need K % 4, tr-form operands M / N % 4; strides % 4.
at::Tensor gemm_f32(const at::Tensor& a, const at::Tensor& b, bool a_tr, bool b_tr, const c10::optional<at::Tensor>& bias,
                    bool relu, double alpha, double beta, const c10::optional<at::Tensor>& out, int64_t splits,
                    int64_t shape) {
  HYP_CHECK_CUDA_TENSOR(a);
  for (const at::Tensor* t : {&a, &b}) {
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->dim() == 2 && t->stride(1) == 1 && t->stride(0) % 4 == 0 &&
                    reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                "gemm_f32: operands must be fp32 2D, unit stride in dim 1, row stride % 4, 16-byte aligned");
  }
  const int M = (int)(a_tr ? a.size(1) : a.size(0)), K = (int)(a_tr ? a.size(0) : a.size(1));
  const int N = (int)(b_tr ? b.size(1) : b.size(0));
  TORCH_CHECK((b_tr ? b.size(0) : b.size(1)) == K, "gemm_f32: reduction extents differ");
  at::Tensor c;
  if (out.has_value()) {
    c = *out;
    TORCH_CHECK(c.scalar_type() == at::kFloat && c.dim() == 2 && c.size(0) == M && c.size(1) == N && c.stride(1) == 1,
                "gemm_f32: out must be fp32 [M, N] with unit column stride");
  } else {
    TORCH_CHECK(beta == 0.0, "gemm_f32: beta != 0 needs out");
    c = at::empty({M, N}, a.options());
  }
  const float* bp = nullptr;
  if (bias.has_value()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() == N, "gemm_f32: bias [N] fp32");
    bp = bias->data_ptr<float>();
  }
  TORCH_CHECK(hyp::gemm_f32_supported(M, N, K, a_tr, b_tr, (int)a.stride(0), (int)b.stride(0), (int)c.stride(0)),
              "gemm_f32: unsupported shape / layout (row-form K % 4, tr-form M / N % 4)");
  const at::DeviceGuard guard(a.device());
  TORCH_CHECK(shape < 5, "gemm_f32: shape 0 (128x128), 1 (256x64), 2 (64x256), 3 (256x128), 4 (128x256) or < 0 (planned)");
  const int sp = hyp::gemm_f32_splits(M, N, K, (int)splits, (int)shape);
  at::Tensor part;
  if (sp > 1) part = at::empty({(int64_t)sp * M * N}, a.options());
  HYP_CHECK_HIP(hyp::gemm_f32(a.data_ptr<float>(), b.data_ptr<float>(), c.data_ptr<float>(),
                              sp > 1 ? part.data_ptr<float>() : nullptr, bp,
                              static_cast<const float*>(device_zero_page(a.device())), M, N, K, a_tr, b_tr,
                              (int)a.stride(0), (int)b.stride(0), (int)c.stride(0), (float)alpha, (float)beta,
                              relu ? 1 : 0, sp, (int)shape, cur_stream()));
  return c;
}

// fp32 a [M, K], b [N, K] -> a @ b.T (the C3 matmul sweep's fp32 row)
at::Tensor gemm_f32_nt(const at::Tensor& a, const at::Tensor& b, c10::optional<at::ScalarType> out_dtype, double alpha) {
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(1), "gemm_f32_nt: expected a [M,K], b [N,K]");
  at::Tensor c = gemm_f32(a, b, false, false, c10::nullopt, false, alpha, 0.0, c10::nullopt, -1, -1);
  return out_dtype.has_value() && *out_dtype != at::kFloat ? c.to(*out_dtype) : c;
}

// x: [N, C, H, W] fp32 channels-last -> cols [N*Ho*Wo, Kp] (Kp >= R*S*C, % 4)
at::Tensor im2col_f32(const at::Tensor& x, int64_t R, int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                      int64_t Kp) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "im2col_f32: fp32 channels-last [N, C, H, W]");
  const int Nb = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int Ho = (int)((H + 2 * ph - R) / sh + 1), Wo = (int)((W + 2 * pw - S) / sw + 1);
  TORCH_CHECK(Kp >= R * S * C && Ho > 0 && Wo > 0, "im2col_f32: bad geometry");
  const at::DeviceGuard guard(x.device());
  auto cols = at::empty({(int64_t)Nb * Ho * Wo, Kp}, x.options());
  HYP_CHECK_HIP(hyp::im2col_f32(x.data_ptr<float>(), cols.data_ptr<float>(), Nb, H, W, C, Ho, Wo, (int)R, (int)S,
                                (int)sh, (int)sw, (int)ph, (int)pw, (int)Kp, cur_stream()));
  return cols;
}

// dcols [N*Ho*Wo, Kp] -> dx [N, C, H, W] fp32 channels-last (the adjoint of im2col_f32)
at::Tensor col2im_f32(const at::Tensor& dcols, int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t R, int64_t S,
                      int64_t sh, int64_t sw, int64_t ph, int64_t pw) {
  HYP_CHECK_CUDA_TENSOR(dcols);
  const int64_t Ho = (H + 2 * ph - R) / sh + 1, Wo = (W + 2 * pw - S) / sw + 1;
  TORCH_CHECK(dcols.scalar_type() == at::kFloat && dcols.dim() == 2 && dcols.is_contiguous() &&
                  dcols.size(0) == Nb * Ho * Wo && dcols.size(1) >= R * S * C,
              "col2im_f32: dcols must be contiguous fp32 [N*Ho*Wo, >= R*S*C]");
  const at::DeviceGuard guard(dcols.device());
  auto dx = at::empty({Nb, C, H, W}, dcols.options().memory_format(at::MemoryFormat::ChannelsLast));
  HYP_CHECK_HIP(hyp::col2im_f32(dcols.data_ptr<float>(), dx.data_ptr<float>(), (int)Nb, (int)H, (int)W, (int)C, (int)Ho,
                                (int)Wo, (int)R, (int)S, (int)sh, (int)sw, (int)ph, (int)pw, (int)dcols.size(1),
                                cur_stream()));
  return dx;
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
  m.def("gemm_f32", &gemm_f32, "C = epi(alpha A·Bᵀ) in fp32 on the fp32-input MFMA (NT/NN/TN, any M/N, split-K)",
        pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("a_tr") = false, pybind11::arg("b_tr") = false,
        pybind11::arg("bias") = pybind11::none(), pybind11::arg("relu") = false, pybind11::arg("alpha") = 1.0,
        pybind11::arg("beta") = 0.0, pybind11::arg("out") = pybind11::none(), pybind11::arg("splits") = -1,
        pybind11::arg("shape") = -1);
  m.def("im2col_f32", &im2col_f32, "NHWC fp32 im2col -> [N*Ho*Wo, Kp]", pybind11::arg("x"), pybind11::arg("R"),
        pybind11::arg("S"), pybind11::arg("sh"), pybind11::arg("sw"), pybind11::arg("ph"), pybind11::arg("pw"),
        pybind11::arg("Kp"));
  m.def("col2im_f32", &col2im_f32, "adjoint of im2col_f32 -> channels-last dx", pybind11::arg("dcols"),
        pybind11::arg("Nb"), pybind11::arg("C"), pybind11::arg("H"), pybind11::arg("W"), pybind11::arg("R"),
        pybind11::arg("S"), pybind11::arg("sh"), pybind11::arg("sw"), pybind11::arg("ph"), pybind11::arg("pw"));
  m.def("gemm_f32_nt", &gemm_f32_nt, "C = alpha * A @ B.T, fp32 in, on the fp32-input MFMA", pybind11::arg("a"),
        pybind11::arg("b"), pybind11::arg("out_dtype") = pybind11::none(), pybind11::arg("alpha") = 1.0);
  m.def("gemm_nt", &gemm_nt, "C = alpha * A @ B.T on MFMA (bf16/f16 in)", pybind11::arg("a"), pybind11::arg("b"),
        pybind11::arg("out_dtype") = pybind11::none(), pybind11::arg("alpha") = 1.0, pybind11::arg("bk") = 64);
}

}  // namespace hypbind
