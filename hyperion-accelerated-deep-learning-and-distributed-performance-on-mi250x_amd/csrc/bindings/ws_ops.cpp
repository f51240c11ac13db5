// Torch bindings: weight-streaming GEMM (kernels/wstream.hip) for the few-token projections of the
// Llama LoRA fine-tune (SURVEY §2.4 "GEMM"/"LoRA", §2.5 Llama row).
#include "bindings/common.h"
#include "bindings/registry.h"

namespace hypbind {
namespace {

struct WsPlan {
  int mf, kr, G, nf, S, MFtot;
};

WsPlan plan_for(int64_t M, int64_t N, int64_t K, bool nn, int64_t mf, int64_t kr, int64_t G, int64_t nf) {
  WsPlan p;
  hyp::ws_plan((int)M, (int)N, (int)K, nn, &p.mf, &p.kr, &p.G, &p.nf);
  if (mf > 0) p.mf = (int)mf;
  if (kr > 0) p.kr = (int)kr;
  if (G > 0) p.G = (int)G;
  if (nf > 0) p.nf = (int)nf;
  p.S = (int)((K + p.kr - 1) / p.kr);
  p.MFtot = (int)((M + p.mf * 16 - 1) / (p.mf * 16)) * p.mf;
  return p;
}

void check_ws(const at::Tensor& x, const at::Tensor& w, bool nn, int64_t* M, int64_t* N, int64_t* K) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.stride(1) == 1 && w.stride(1) == 1, "ws: 2D operands, unit column stride");
  TORCH_CHECK(x.scalar_type() == w.scalar_type() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf),
              "ws: bf16/f16 operands of one dtype");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "ws: 16-byte aligned rows");
  *M = x.size(0);
  *K = x.size(1);
  *N = nn ? w.size(1) : w.size(0);
  TORCH_CHECK((nn ? w.size(0) : w.size(1)) == *K, "ws: reduction sizes differ");
  TORCH_CHECK(hyp::ws_supported((int)*M, (int)*N, (int)*K, nn),
              "ws: unsupported shape (K % 32, N % 16 (NT) / N % 64 (NN))");
}

// fp32 partial slabs of x·Wᵀ (nn = false) / x·W (nn = true) -> (part, S, MFtot)
std::tuple<at::Tensor, int64_t, int64_t> ws_gemm_part(const at::Tensor& x, const at::Tensor& w, bool nn, int64_t mf,
                                                      int64_t kr, int64_t G, int64_t nf, bool slab16) {
  int64_t M, N, K;
  check_ws(x, w, nn, &M, &N, &K);
  const WsPlan p = plan_for(M, N, K, nn, mf, kr, G, nf);
  const at::DeviceGuard guard(x.device());
  auto part = at::empty({(int64_t)p.S * p.MFtot * (N / 16) * 256}, x.options().dtype(slab16 ? at::kBFloat16 : at::kFloat));
  HYP_CHECK_HIP(hyp::ws_gemm(dtype_code(x), nn, x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0),
                             static_cast<float*>(part.data_ptr()), device_zero_page(x.device()), (int)M, (int)N, (int)K,
                             p.mf, p.kr, p.G, p.nf, cur_stream(), slab16 ? 1 : 0));
  return {part, p.S, p.MFtot};
}

// slab buffer -> (pointer, bf16 flag)
std::pair<const float*, int> slab_ptr(const at::Tensor& part, int64_t need, const char* what) {
  TORCH_CHECK(part.is_cuda() && part.is_contiguous() && part.numel() >= need &&
                  (part.scalar_type() == at::kFloat || part.scalar_type() == at::kBFloat16),
              what, ": fp32 or bf16 slabs of the weight-streaming GEMM");
  return {static_cast<const float*>(part.data_ptr()), part.scalar_type() == at::kBFloat16 ? 1 : 0};
}

at::Tensor ws_reduce(const at::Tensor& part, int64_t M, int64_t N, int64_t S, int64_t MFtot, bool nn,
                     at::ScalarType dtype, double alpha, const c10::optional<at::Tensor>& addend, double beta,
                     const c10::optional<at::Tensor>& U, const c10::optional<at::Tensor>& V, int64_t segw,
                     double uscale, const c10::optional<at::Tensor>& out) {
  const auto sp = slab_ptr(part, S * MFtot * (N / 16) * 256, "ws_reduce");
  TORCH_CHECK(MFtot * 16 >= M, "ws_reduce: MFtot too small");
  const at::DeviceGuard guard(part.device());
  at::Tensor o;
  if (out.has_value() && out->defined()) {
    o = *out;
    TORCH_CHECK(o.dim() == 2 && o.size(0) == M && o.size(1) == N && o.stride(1) == 1 && o.scalar_type() == dtype,
                "ws_reduce: out must be [M, N] in the output dtype");
  } else {
    o = at::empty({M, N}, part.options().dtype(dtype));
  }
  const void* add = nullptr;
  if (addend.has_value() && addend->defined()) {
    TORCH_CHECK(addend->sizes() == o.sizes() && addend->stride(0) == o.stride(0) && addend->stride(1) == 1 &&
                    addend->scalar_type() == dtype,
                "ws_reduce: addend like out");
    add = addend->data_ptr();
  }
  const float* u = nullptr;
  const void* v = nullptr;
  int r = 0;
  if (U.has_value() && U->defined()) {
    TORCH_CHECK(V.has_value() && V->defined(), "ws_reduce: U needs V");
    TORCH_CHECK(U->scalar_type() == at::kFloat && U->is_contiguous() && U->size(0) == M, "ws_reduce: U fp32 [M, nseg*r]");
    TORCH_CHECK(V->scalar_type() == dtype && V->is_contiguous() && V->size(0) == N, "ws_reduce: V [N, r] in out dtype");
    TORCH_CHECK(segw > 0 && N % segw == 0 && U->size(1) == (N / segw) * V->size(1), "ws_reduce: segments");
    u = U->data_ptr<float>();
    v = V->data_ptr();
    r = (int)V->size(1);
  }
  HYP_CHECK_HIP(hyp::ws_reduce(dtype == at::kBFloat16 ? hyp::kBF16 : hyp::kF16, nn, sp.first,
                               o.data_ptr(), o.stride(0), add, (float)alpha, (float)beta, u, v, r, (int)segw,
                               (float)uscale, (int)M, (int)N, (int)S, (int)MFtot, cur_stream(), sp.second));
  return o;
}

at::Tensor ws_linear(const at::Tensor& x, const at::Tensor& w, bool nn, double alpha,
                     const c10::optional<at::Tensor>& addend, double beta, int64_t mf, int64_t kr, int64_t G,
                     int64_t nf) {
  auto res = ws_gemm_part(x, w, nn, mf, kr, G, nf, false);
  const int64_t M = x.size(0), N = nn ? w.size(1) : w.size(0);
  return ws_reduce(std::get<0>(res), M, N, std::get<1>(res), std::get<2>(res), nn, x.scalar_type(), alpha, addend,
                   beta, c10::nullopt, c10::nullopt, 1, 1.0, c10::nullopt);
}

std::vector<int64_t> ws_plan_py(int64_t M, int64_t N, int64_t K, bool nn) {
  const WsPlan p = plan_for(M, N, K, nn, 0, 0, 0, 0);
  return {p.mf, p.kr, p.G, p.nf, p.S, p.MFtot};
}


// ---- fused epilogues + LoRA rank-r kernels (ops/llama_fused.py) ------------------------------
void check_out(const at::Tensor& o, int64_t M, int64_t N, at::ScalarType dt, const char* what) {
  TORCH_CHECK(o.is_cuda() && o.dim() == 2 && o.size(0) == M && o.size(1) == N && o.stride(1) == 1 &&
                  o.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(o.data_ptr()) % 16 == 0 && o.scalar_type() == dt,
              "ws_epilogue: ", what, " must be [", M, ", ", N, "] row-major (16-byte rows) in the activation dtype");
}

std::vector<const void*> ptr_list(const std::vector<at::Tensor>& ts, at::ScalarType dt, const char* what) {
  std::vector<const void*> v;
  for (const auto& t : ts) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == dt, what, ": contiguous tensors in the activation dtype");
    v.push_back(t.data_ptr());
  }
  return v;
}

// A rank-r fp32 buffer: [M, >= W] (one slice) or a split-partial stack [S, M, >= W] (slices summed by
// the consumer); unit stride in the last dim.
struct RankRView {
  float* p;
  int ld, S;
  int64_t sstride;
};

RankRView rank_r_view(const at::Tensor& t, int64_t M, int64_t W, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && (t.dim() == 2 || t.dim() == 3) && t.stride(-1) == 1,
              what, ": fp32 [M, W] or [splits, M, W] with unit stride in the last dim");
  TORCH_CHECK(t.size(-2) == M && t.size(-1) >= W, what, ": shape must be [.., M, >= ", W, "]");
  RankRView v;
  v.p = t.data_ptr<float>();
  v.ld = (int)t.stride(-2);
  v.S = t.dim() == 3 ? (int)t.size(0) : 1;
  v.sstride = t.dim() == 3 ? t.stride(0) : 0;
  return v;
}

void ws_epilogue_py(const c10::optional<at::Tensor>& part_opt, int64_t S, int64_t MFtot, int64_t M, int64_t N, int64_t epi,
                    const at::Tensor& out, const c10::optional<at::Tensor>& out2, const c10::optional<at::Tensor>& aux,
                    const c10::optional<at::Tensor>& t, const std::vector<at::Tensor>& lw, int64_t segw, double lscale,
                    int64_t rope_segs, int64_t seq, double theta, const c10::optional<at::Tensor>& rng, double p_drop,
                    c10::optional<bool> nn, const c10::optional<at::Tensor>& yin) {
  const bool dense = !(part_opt.has_value() && part_opt->defined());
  const float* part_ptr = nullptr;
  int sb = 0;
  if (!dense) {
    const auto sp = slab_ptr(*part_opt, S * MFtot * (N / 16) * 256, "ws_epilogue");
    part_ptr = sp.first;
    sb = sp.second;
  } else {
    TORCH_CHECK(yin.has_value() && yin->defined() && yin->dim() == 2 && yin->size(0) == M && yin->size(1) == N &&
                    yin->stride(1) == 1 && yin->scalar_type() == out.scalar_type(),
                "ws_epilogue: without slabs, yin must be the [M, N] GEMM result in the activation dtype");
    MFtot = (M + 15) / 16;
    S = 0;
  }
  const auto dt = out.scalar_type();
  const int64_t I = N;  // EPI 2: out is gu [M, N], out2 h [M, N/2]; EPI 3: out is dgu [M, 2N]
  check_out(out, M, epi == 3 ? 2 * N : N, dt, "out");
  void* o2 = nullptr;
  int64_t ldo2 = 0;
  if (epi == 2) {
    TORCH_CHECK(out2.has_value() && out2->defined(), "ws_epilogue: SwiGLU needs out2 (h)");
    check_out(*out2, M, I / 2, dt, "out2");
    o2 = out2->data_ptr();
    ldo2 = out2->stride(0);
  }
  const void* ax = nullptr;
  int64_t ldax = 0;
  if (epi == 3) {
    TORCH_CHECK(aux.has_value() && aux->defined(), "ws_epilogue: SwiGLU backward needs gu");
    check_out(*aux, M, 2 * N, dt, "aux (gu)");
    ax = aux->data_ptr();
    ldax = aux->stride(0);
  }
  const float* tp = nullptr;
  int ldt = 0, r = 0, P = 0, t_S = 1;
  int64_t t_ss = 0;
  std::vector<const void*> lp;
  if (epi == 4 || (epi == 1 && t.has_value() && t->defined())) {
    TORCH_CHECK(t.has_value() && t->defined(), "ws_epilogue: this epilogue needs t");
    lp = ptr_list(lw, dt, "ws_epilogue lw");
    P = (int)lw.size();
    TORCH_CHECK(P >= 1 && P <= 4, "ws_epilogue: 1..4 LoRA projections");
    r = (int)(epi == 1 ? lw[0].size(1) : lw[0].size(0));
    for (const auto& w : lw)
      TORCH_CHECK(epi == 1 ? (w.size(1) == r && w.size(0) == segw) : (w.size(0) == r && w.size(1) == N),
                  "ws_epilogue: LoRA operand shapes (B_p [segw, r] / A_p [r, N])");
    const RankRView tv = rank_r_view(*t, M, P * r, "ws_epilogue t");
    tp = tv.p;
    ldt = tv.ld;
    t_ss = tv.sstride;
    t_S = tv.S;
  }
  hyp::RngState rs{};
  const bool has_rng = rng.has_value() && rng->defined() && p_drop > 0;
  if (has_rng) rs = unpack_rng(*rng);
  TORCH_CHECK(epi != 1 || (segw >= 128 && N % segw == 0), "ws_epilogue: segment width");
  const at::DeviceGuard guard(out.device());
  HYP_CHECK_HIP(hyp::ws_epilogue(dtype_code(out), (int)epi, part_ptr, (int)S, (int)MFtot, (int)M,
                                 (int)N, out.data_ptr(), out.stride(0), o2, ldo2, ax, ldax, tp, ldt, t_ss, t_S,
                                 lp.empty() ? nullptr : lp.data(), P, r, (int)segw, (float)lscale, (int)rope_segs,
                                 (int)seq, (float)theta, has_rng ? &rs : nullptr, (float)p_drop,
                                 nn.has_value() ? *nn : (epi == 3 || epi == 4), dense ? yin->data_ptr() : nullptr,
                                 dense ? yin->stride(0) : 0, cur_stream(), sb));
}

void lora_down_py(const at::Tensor& x, const std::vector<at::Tensor>& A, at::Tensor& t,
                  const c10::optional<at::Tensor>& rng, double p_drop) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "lora_down: x [M, K] row-major");
  auto lp = ptr_list(A, x.scalar_type(), "lora_down A");
  const int P = (int)A.size(), r = (int)A[0].size(0);
  for (const auto& a : A) TORCH_CHECK(a.dim() == 2 && a.size(0) == r && a.size(1) == x.size(1), "lora_down: A_p [r, K]");
  const RankRView tv = rank_r_view(t, x.size(0), P * r, "lora_down t");
  hyp::RngState rs{};
  const bool has_rng = rng.has_value() && rng->defined() && p_drop > 0;
  if (has_rng) rs = unpack_rng(*rng);
  const at::DeviceGuard guard(x.device());
  HYP_CHECK_HIP(hyp::lora_down(dtype_code(x), x.data_ptr(), x.stride(0), lp.data(), P, r, tv.p, tv.ld, tv.sstride, tv.S,
                               (int)x.size(0), (int)x.size(1), has_rng ? &rs : nullptr, (float)p_drop, cur_stream()));
}

void lora_bwd_t_py(const at::Tensor& dy, int64_t N, const std::vector<at::Tensor>& B, const std::vector<at::Tensor>& dB,
                   const at::Tensor& t, at::Tensor& du, double c) {
  HYP_CHECK_CUDA_TENSOR(dy);
  TORCH_CHECK(dy.dim() == 2 && dy.stride(1) == 1 && dy.size(1) >= (int64_t)B.size() * N, "lora_bwd_t: dy [M, >= P N]");
  auto bp = ptr_list(B, dy.scalar_type(), "lora_bwd_t B");
  auto dbp = ptr_list(dB, dy.scalar_type(), "lora_bwd_t dB");
  TORCH_CHECK(B.size() == dB.size(), "lora_bwd_t: B / dB lists differ");
  const int P = (int)B.size(), r = (int)B[0].size(1);
  for (size_t i = 0; i < B.size(); ++i)
    TORCH_CHECK(B[i].size(0) == N && B[i].size(1) == r && dB[i].sizes() == B[i].sizes(), "lora_bwd_t: B_p [N, r]");
  const RankRView tv = rank_r_view(t, dy.size(0), P * r, "lora_bwd_t t");
  const RankRView uv = rank_r_view(du, dy.size(0), P * r, "lora_bwd_t du");
  std::vector<void*> dbw;
  for (auto* q : dbp) dbw.push_back(const_cast<void*>(q));
  const at::DeviceGuard guard(dy.device());
  HYP_CHECK_HIP(hyp::lora_bwd_t(dtype_code(dy), dy.data_ptr(), dy.stride(0), (int)N, bp.data(), dbw.data(), P, r, tv.p,
                                tv.ld, tv.sstride, tv.S, uv.p, uv.ld, uv.sstride, uv.S, (int)dy.size(0), (float)c,
                                cur_stream()));
}

void lora_bwd_a_py(const at::Tensor& x, const std::vector<at::Tensor>& dA, const at::Tensor& du,
                   const c10::optional<at::Tensor>& rng, double p_drop) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "lora_bwd_a: x [M, K] row-major");
  auto dap = ptr_list(dA, x.scalar_type(), "lora_bwd_a dA");
  const int P = (int)dA.size(), r = (int)dA[0].size(0);
  for (const auto& a : dA) TORCH_CHECK(a.size(0) == r && a.size(1) == x.size(1), "lora_bwd_a: dA_p [r, K]");
  const RankRView uv = rank_r_view(du, x.size(0), P * r, "lora_bwd_a du");
  std::vector<void*> daw;
  for (auto* q : dap) daw.push_back(const_cast<void*>(q));
  hyp::RngState rs{};
  const bool has_rng = rng.has_value() && rng->defined() && p_drop > 0;
  if (has_rng) rs = unpack_rng(*rng);
  const at::DeviceGuard guard(x.device());
  HYP_CHECK_HIP(hyp::lora_bwd_a(dtype_code(x), x.data_ptr(), x.stride(0), (int)x.size(1), daw.data(), P, r, uv.p, uv.ld,
                                uv.sstride, uv.S, (int)x.size(0), has_rng ? &rs : nullptr, (float)p_drop, cur_stream()));
}
}  // namespace

void register_ws_ops(pybind11::module& m) {
  using namespace pybind11::literals;
  m.def("ws_gemm_part", &ws_gemm_part,
        "weight-streaming GEMM -> (fragment-order partial slabs: fp32, or bf16 with slab16, S, MFtot)", "x"_a, "w"_a,
        "nn"_a = false, "mf"_a = 0, "kr"_a = 0, "G"_a = 0, "nf"_a = 0, "slab16"_a = false);
  m.def("ws_reduce", &ws_reduce, "sum weight-streaming partial slabs (+ alpha, addend, rank-r term)", "part"_a, "M"_a,
        "N"_a, "S"_a, "MFtot"_a, "nn"_a, "dtype"_a, "alpha"_a = 1.0, "addend"_a = pybind11::none(), "beta"_a = 1.0,
        "U"_a = pybind11::none(), "V"_a = pybind11::none(), "segw"_a = 1, "uscale"_a = 1.0, "out"_a = pybind11::none());
  m.def("ws_linear", &ws_linear, "y = alpha x Wᵀ (nn=False) / alpha x W (nn=True) (+ beta addend)", "x"_a, "w"_a,
        "nn"_a = false, "alpha"_a = 1.0, "addend"_a = pybind11::none(), "beta"_a = 1.0, "mf"_a = 0, "kr"_a = 0,
        "G"_a = 0, "nf"_a = 0);
  m.def("ws_plan", &ws_plan_py, "(mf, kr, G, nf, S, MFtot) of the automatic plan");
  m.def("ws_set_depth", [](int64_t d) { hyp::ws_set_depth((int)d); },
        "weight-streaming GEMM: k-steps in flight per wave (4 default, 8 where the slices allow)");
  m.def("ws_epilogue", &ws_epilogue_py, "fused slab epilogue (0 plain, 1 LoRA up + RoPE, 2 SwiGLU, 3 SwiGLU bwd, 4 LoRA dgrad)",
        "part"_a, "S"_a, "MFtot"_a, "M"_a, "N"_a, "epi"_a, "out"_a, "out2"_a = pybind11::none(),
        "aux"_a = pybind11::none(), "t"_a = pybind11::none(), "lw"_a = std::vector<at::Tensor>{}, "segw"_a = 0,
        "lscale"_a = 1.0, "rope_segs"_a = 0, "seq"_a = 0, "theta"_a = 10000.0, "rng"_a = pybind11::none(),
        "p_drop"_a = 0.0, "nn"_a = pybind11::none(), "yin"_a = pybind11::none());
  m.def("lora_down", &lora_down_py,
        "t[m, p r + j] = Σ_k keep_p x A_p; t [M, W] or a k-split partial stack [S, M, W] (slice q = split q)", "x"_a,
        "A"_a, "t"_a, "rng"_a = pybind11::none(), "p_drop"_a = 0.0);
  m.def("lora_bwd_t", &lora_bwd_t_py, "du' = c dy_p B_p (n-split partial stack if du is 3D); dB_p = c dy_pᵀ t_p (t: stack summed)", "dy"_a, "N"_a, "B"_a, "dB"_a,
        "t"_a, "du"_a, "c"_a);
  m.def("lora_bwd_a", &lora_bwd_a_py, "dA_p = du'_pᵀ (keep_p ∘ x)", "x"_a, "dA"_a, "du"_a, "rng"_a = pybind11::none(),
        "p_drop"_a = 0.0);
}

}  // namespace hypbind
