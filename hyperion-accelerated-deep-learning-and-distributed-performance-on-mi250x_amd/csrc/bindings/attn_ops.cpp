// Torch bindings: flash attention fwd/bwd and LayerNorm/RMSNorm fwd/bwd.
#include <cmath>
#include "bindings/common.h"
#include "bindings/registry.h"

namespace hypbind {
namespace {

// attn_set_qsplit: 0 = automatic query split of the S <= 128 backward, 1 = off, n > 1 = at most n
int g_attn_qsplit = 0;


void check_bshd(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4, name, " must be a [B,S,H,D] GPU tensor");
  TORCH_CHECK(t.stride(3) == 1, name, " must have a contiguous head dim");
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0,
              name, " strides must be multiples of 8 elements (16-byte vector loads)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

std::vector<at::Tensor> attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, bool causal,
                                 double scale, double p_drop, const c10::optional<at::Tensor>& rng, const c10::optional<at::Tensor>& kpm,
                                 bool need_lse) {
  check_bshd(q, "q");
  check_bshd(k, "k");
  check_bshd(v, "v");
  TORCH_CHECK(q.sizes() == k.sizes() && q.sizes() == v.sizes(), "attn_fwd: self-attention shapes must match");
  const int B = q.size(0), S = q.size(1), H = q.size(2), D = q.size(3);
  const int dt = dtype_code(q);
  TORCH_CHECK(hyp::attention_supported(dt, D), "attn_fwd: needs bf16/fp16 and head_dim 64 or 128");
  const at::DeviceGuard guard(q.device());
  auto o = at::empty({B, S, H, D}, q.options());
  at::Tensor lse;
  if (need_lse) lse = at::empty({B * H, S}, q.options().dtype(at::kFloat));
  at::Tensor kpm_u8;
  if (kpm.has_value() && kpm->defined()) {
    kpm_u8 = kpm->to(at::kByte).contiguous();
    TORCH_CHECK(kpm_u8.size(0) == B && kpm_u8.size(1) == S, "key_padding_mask must be [B, S]");
  }
  hyp::AttnParams p{};
  p.q = q.data_ptr(); p.k = k.data_ptr(); p.v = v.data_ptr(); p.o = o.data_ptr();
  p.sqb = q.stride(0); p.sqs = q.stride(1); p.sqh = q.stride(2);
  p.skb = k.stride(0); p.sks = k.stride(1); p.skh = k.stride(2);
  p.svb = v.stride(0); p.svs = v.stride(1); p.svh = v.stride(2);
  p.sob = o.stride(0); p.sos = o.stride(1); p.soh = o.stride(2);
  p.lse = need_lse ? lse.data_ptr<float>() : nullptr;
  p.kpm = kpm_u8.defined() ? kpm_u8.data_ptr<uint8_t>() : nullptr;
  p.B = B; p.H = H; p.S = S; p.D = D;
  p.scale_log2 = (float)(scale * 1.4426950408889634);
  p.causal = causal ? 1 : 0;
  p.p_drop = (float)p_drop;
  if (p_drop > 0) {
    TORCH_CHECK(rng.has_value() && rng->defined(), "attention dropout needs an rng state (hyperion._C.rng_state)");
    p.rng = unpack_rng(*rng);
  } else {
    p.rng = hyp::RngState{};
  }
  HYP_CHECK_HIP(hyp::attention_forward(dt, p, cur_stream()));
  return {o, lse};
}

// grads are written into dq/dk/dv (any [B,S,H,D] strided views, e.g. slices of a packed dQKV)
void attn_bwd_impl(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                   const at::Tensor& o, const at::Tensor& lse, bool causal, double scale, double p_drop,
                   const c10::optional<at::Tensor>& rng, const c10::optional<at::Tensor>& kpm, at::Tensor& dq,
                   at::Tensor& dk, at::Tensor& dv, const at::Tensor* rope_cs) {
  check_bshd(q, "q");
  check_bshd(k, "k");
  check_bshd(v, "v");
  check_bshd(o, "o");
  check_bshd(dq, "dq");
  check_bshd(dk, "dk");
  check_bshd(dv, "dv");
  at::Tensor g = dout.stride(3) == 1 && dout.stride(0) % 8 == 0 && dout.stride(1) % 8 == 0 && dout.stride(2) % 8 == 0
                     ? dout
                     : dout.contiguous();
  check_bshd(g, "dout");
  const int B = q.size(0), S = q.size(1), H = q.size(2), D = q.size(3);
  const int dt = dtype_code(q);
  const at::DeviceGuard guard(q.device());
  auto fopt = q.options().dtype(at::kFloat);
  auto delta = at::empty({(int64_t)B * H * S}, fopt);
  // fp32 dQ workspace only when several key blocks add into one dQ row (attn_bwd_k stores dQ
  // directly for S <= 128)
  at::Tensor dq_acc;
  // 2-4 key blocks (ViT-B/16's 197 tokens): one fp32 slab per key block, summed in order by the
  // conversion pass (deterministic, no zero-fill, no atomics); more blocks: fp32 atomics
  const int nkb = (S + 127) / 128;
  const int dq_slabs = (nkb >= 2 && nkb <= 4) ? nkb : 0;
  if (S > 128) dq_acc = at::empty({(int64_t)(dq_slabs ? dq_slabs : 1) * B * H * S * D}, fopt);
  // S <= 128 with few (b, h) pairs (Llama-2-7B at batch 1: 32 heads = 32 workgroups on 256 CUs):
  // split each head's query slices over qsplit workgroups; dK / dV come back as fp32 partials
  // summed in order by one small pass (dQ of a slice is still complete in its workgroup)
  int qsplit = 1;
  at::Tensor dkv_part;
  if (S <= 128 && g_attn_qsplit != 1) {
    const int nsl = (S + (4096 / D) - 1) / (4096 / D);
    const int cap = g_attn_qsplit > 1 ? g_attn_qsplit : nsl;
    // up to 128 workgroups (GPT-2's 192 (b, h) pairs measured no better split: the partial-sum pass
    // costs what the wider grid saves)
    while ((int64_t)B * H * qsplit < 128 && qsplit * 2 <= nsl && qsplit * 2 <= cap) qsplit *= 2;
    if (qsplit > 1) dkv_part = at::empty({(int64_t)qsplit * 2 * B * H * S * D}, fopt);
  }
  at::Tensor kpm_u8;
  if (kpm.has_value() && kpm->defined()) kpm_u8 = kpm->to(at::kByte).contiguous();
  hyp::AttnBwdParams p{};
  p.qsplit = qsplit;
  p.dkv_part = dkv_part.defined() ? dkv_part.data_ptr<float>() : nullptr;
  p.q = q.data_ptr(); p.k = k.data_ptr(); p.v = v.data_ptr(); p.o = o.data_ptr(); p.dout = g.data_ptr();
  p.dq = dq.data_ptr(); p.dk = dk.data_ptr(); p.dv = dv.data_ptr();
  p.sqb = q.stride(0); p.sqs = q.stride(1); p.sqh = q.stride(2);
  p.skb = k.stride(0); p.sks = k.stride(1); p.skh = k.stride(2);
  p.svb = v.stride(0); p.svs = v.stride(1); p.svh = v.stride(2);
  p.sob = o.stride(0); p.sos = o.stride(1); p.soh = o.stride(2);
  p.sdob = g.stride(0); p.sdos = g.stride(1); p.sdoh = g.stride(2);
  p.sdqb = dq.stride(0); p.sdqs = dq.stride(1); p.sdqh = dq.stride(2);
  p.sdkb = dk.stride(0); p.sdks = dk.stride(1); p.sdkh = dk.stride(2);
  p.sdvb = dv.stride(0); p.sdvs = dv.stride(1); p.sdvh = dv.stride(2);
  p.lse = lse.data_ptr<float>();
  p.delta = delta.data_ptr<float>();
  p.dq_acc = dq_acc.defined() ? dq_acc.data_ptr<float>() : nullptr;
  p.dq_slabs = dq_acc.defined() ? dq_slabs : 0;
  p.kpm = kpm_u8.defined() ? kpm_u8.data_ptr<uint8_t>() : nullptr;
  p.B = B; p.H = H; p.S = S; p.D = D;
  p.scale = (float)scale;
  p.scale_log2 = (float)(scale * 1.4426950408889634);
  p.causal = causal ? 1 : 0;
  p.p_drop = (float)p_drop;
  if (p_drop > 0) {
    TORCH_CHECK(rng.has_value() && rng->defined(), "attention dropout needs an rng state (hyperion._C.rng_state)");
    p.rng = unpack_rng(*rng);
  } else {
    p.rng = hyp::RngState{};
  }
  p.rope = rope_cs != nullptr ? 1 : 0;
  p.rope_cs = nullptr;
  if (rope_cs != nullptr) {
    TORCH_CHECK(D == 128 && p_drop == 0, "attn_bwd_rope: head_dim 128 without dropout");
    TORCH_CHECK(rope_cs->is_cuda() && rope_cs->scalar_type() == at::kFloat && rope_cs->is_contiguous() &&
                    rope_cs->numel() >= (int64_t)S * 128,
                "attn_bwd_rope: table must be fp32 [>= S, 64, 2] (cos, sin)");
    p.rope_cs = reinterpret_cast<const float2*>(rope_cs->data_ptr<float>());
  }
  HYP_CHECK_HIP(hyp::attention_backward(dt, p, cur_stream()));
}

void attn_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
              const at::Tensor& o, const at::Tensor& lse, bool causal, double scale, double p_drop, const c10::optional<at::Tensor>& rng,
              const c10::optional<at::Tensor>& kpm, at::Tensor& dq, at::Tensor& dk, at::Tensor& dv) {
  attn_bwd_impl(dout, q, k, v, o, lse, causal, scale, p_drop, rng, kpm, dq, dk, dv, nullptr);
}

// the same, with dQ / dK leaving through the inverse rotary embedding (positions = sequence index;
// cs = the (cos, sin) table [S, 64, 2] of ops.rope.rope_table)
void attn_bwd_rope(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                   const at::Tensor& o, const at::Tensor& lse, bool causal, double scale,
                   const c10::optional<at::Tensor>& kpm, at::Tensor& dq, at::Tensor& dk, at::Tensor& dv,
                   const at::Tensor& cs) {
  attn_bwd_impl(dout, q, k, v, o, lse, causal, scale, 0.0, c10::nullopt, kpm, dq, dk, dv, &cs);
}

// ---- LayerNorm / RMSNorm ------------------------------------------------------------------
// affine parameters: fp32, or (wt = 1) the activation dtype; weight and bias must agree
int affine_mode(const at::Tensor& x, const c10::optional<at::Tensor>& w, const c10::optional<at::Tensor>& b,
                const char* what) {
  int mode = -1;
  for (const auto* t : {&w, &b}) {
    if (!t->has_value() || !(*t)->defined()) continue;
    const at::Tensor& a = **t;
    TORCH_CHECK(a.is_contiguous() && a.device() == x.device() && a.numel() == x.size(-1), what,
                ": affine parameter must be a contiguous [d] tensor on the input's device");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0, what, ": affine parameter must be 16-byte aligned");
    const int m = a.scalar_type() == at::kFloat ? 0 : (a.scalar_type() == x.scalar_type() ? 1 : -2);
    TORCH_CHECK(m >= 0, what, ": affine parameters must be fp32 or the input dtype");
    TORCH_CHECK(mode < 0 || mode == m, what, ": weight and bias dtypes differ");
    mode = m;
  }
  return mode < 0 ? 0 : mode;
}

const float* affine_ptr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? static_cast<const float*>(t->data_ptr()) : nullptr;
}

// x: [..., d] contiguous; returns (y, s (fused residual stream or undefined), mean, rstd)
// drop_p > 0 (with a residual and the rng record of ops._native.rng_state): s = residual + dropout(x)
std::vector<at::Tensor> ln_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& residual,
                               const c10::optional<at::Tensor>& weight, const c10::optional<at::Tensor>& bias,
                               double eps, bool rms, double drop_p, const c10::optional<at::Tensor>& rng) {
  HYP_CHECK_CUDA_TENSOR(x);
  TORCH_CHECK(x.is_contiguous(), "ln_fwd: x must be contiguous");
  const int d = x.size(-1);
  TORCH_CHECK(hyp::layernorm_supported(d), "ln_fwd: unsupported hidden size ", d);
  const int64_t rows = x.numel() / d;
  const at::DeviceGuard guard(x.device());
  auto y = at::empty_like(x);
  at::Tensor s;
  const bool has_res = residual.has_value() && residual->defined();
  if (has_res) {
    TORCH_CHECK(residual->is_contiguous() && residual->sizes() == x.sizes() &&
                    residual->scalar_type() == x.scalar_type(),
                "ln_fwd: residual mismatch");
    s = at::empty_like(x);
  }
  auto fopt = x.options().dtype(at::kFloat);
  auto mean = at::empty({rows}, fopt);
  auto rstd = at::empty({rows}, fopt);
  const int wt = affine_mode(x, weight, bias, "ln_fwd");
  hyp::RngState rs{};
  if (drop_p > 0.0) {
    TORCH_CHECK(has_res && d <= 2048 && drop_p < 1.0 && rng.has_value() && rng->defined(),
                "ln_fwd: dropout needs a residual, d <= 2048, p < 1 and an rng record");
    rs = unpack_rng(*rng);
  }
  HYP_CHECK_HIP(hyp::layernorm_forward(dtype_code(x), rms ? 1 : 0, x.data_ptr(), has_res ? residual->data_ptr() : nullptr,
                                       has_res ? s.data_ptr() : nullptr, y.data_ptr(), affine_ptr(weight),
                                       affine_ptr(bias), rms ? nullptr : mean.data_ptr<float>(),
                                       rstd.data_ptr<float>(), rows, d, (float)eps, cur_stream(), wt, (float)drop_p,
                                       drop_p > 0.0 ? &rs : nullptr));
  return {y, s, mean, rstd};
}

// returns (dx, dweight, dbias, dxa): dxa = dropout(dx) with the forward's mask when drop_p > 0
std::vector<at::Tensor> ln_bwd(const at::Tensor& dy, const at::Tensor& xin, const c10::optional<at::Tensor>& weight,
                               const at::Tensor& mean, const at::Tensor& rstd, const c10::optional<at::Tensor>& dres,
                               bool need_dw, bool need_db, bool rms, double drop_p,
                               const c10::optional<at::Tensor>& rng, bool branch_sum, int64_t bsum_dtype) {
  const int d = xin.size(-1);
  const int64_t rows = xin.numel() / d;
  at::Tensor g = dy.is_contiguous() ? dy : dy.contiguous();
  const at::DeviceGuard guard(xin.device());
  auto dx = at::empty_like(xin);
  int P = 1, rpw = 1;
  hyp::layernorm_bwd_geom(rows, d, &P, &rpw);
  auto fopt = xin.options().dtype(at::kFloat);
  branch_sum = branch_sum && d <= 2048;
  auto part = at::empty({(branch_sum ? 3 : 2) * (int64_t)P * d}, fopt);
  const int wt = affine_mode(xin, weight, c10::nullopt, "ln_bwd");
  auto wopt = wt ? xin.options() : fopt;  // dγ / dβ in the weight's dtype
  // LayerNorm: dγ and dβ come out of one combine pass into one [2, d] buffer (both computed)
  at::Tensor dw, db, dwdb, dbs;
  // bsum_dtype (>= 0, a DTYPE_CODE): the branch sums in the consuming linear's bias dtype, their own
  // buffer written by the same combine (no cast kernel after it when the norm keeps fp32 weights)
  const bool own_bs = branch_sum && bsum_dtype >= 0 && bsum_dtype != dtype_code(wopt.dtype().toScalarType());
  if (own_bs) {
    dwdb = at::empty({rms ? 1 : 2, d}, wopt);
    dw = dwdb[0];
    if (!rms) db = dwdb[1];
    dbs = at::empty({d}, xin.options().dtype(scalar_of_code(bsum_dtype)));
  } else if (branch_sum) {  // [dγ | dβ | Σ branch gradient] (RMS: [dγ | Σ]) from one combine
    dwdb = at::empty({rms ? 2 : 3, d}, wopt);
    dw = dwdb[0];
    if (!rms) db = dwdb[1];
    dbs = dwdb[rms ? 1 : 2];
  } else if (!rms && (need_dw || need_db)) {
    dwdb = at::empty({2, d}, wopt);
    dw = dwdb[0];
    db = dwdb[1];
  } else if (need_dw) {
    dw = at::empty({d}, wopt);
  }
  at::Tensor dr;
  if (dres.has_value() && dres->defined()) dr = dres->is_contiguous() ? *dres : dres->contiguous();
  hyp::RngState rs{};
  at::Tensor dxa;
  if (drop_p > 0.0) {
    TORCH_CHECK(d <= 2048 && drop_p < 1.0 && rng.has_value() && rng->defined(),
                "ln_bwd: dropout needs d <= 2048, p < 1 and the forward's rng record");
    rs = unpack_rng(*rng);
    dxa = at::empty_like(xin);
  }
  HYP_CHECK_HIP(hyp::layernorm_backward(dtype_code(xin), rms ? 1 : 0, g.data_ptr(), xin.data_ptr(),
                                        affine_ptr(weight), rms ? nullptr : mean.data_ptr<float>(),
                                        rstd.data_ptr<float>(), dr.defined() ? dr.data_ptr() : nullptr, dx.data_ptr(),
                                        part.data_ptr<float>(), db.defined() ? part.data_ptr<float>() + d : nullptr,
                                        dw.defined() ? dw.data_ptr() : nullptr, db.defined() ? db.data_ptr() : nullptr,
                                        rows, d, P, rpw, cur_stream(), wt, dxa.defined() ? dxa.data_ptr() : nullptr,
                                        (float)drop_p, drop_p > 0.0 ? &rs : nullptr,
                                        dbs.defined() ? dbs.data_ptr() : nullptr, own_bs ? (int)bsum_dtype : -1));
  return {dx, need_dw ? dw : at::Tensor(), need_db ? db : at::Tensor(), dxa, dbs};
}

}  // namespace

void register_attn_ops(pybind11::module& m) {
  m.def("attn_fwd", &attn_fwd, "flash attention forward (MFMA)");
  m.def("attn_bwd", &attn_bwd, "flash attention backward (MFMA)");
  m.def("attn_set_fwd_narrow", [](int64_t on) { hyp::attn_set_fwd_narrow((int)on); },
        "attention forward: one-wave workgroups for grids below 128 workgroups (A/B; default off)");
  m.def("attn_set_qsplit", [](int64_t n) { g_attn_qsplit = (int)n; },
        "S <= 128 attention backward: 0 automatic query split, 1 off, n > 1 at most n (A/B)");
  m.def("attn_bwd_rope", &attn_bwd_rope, "flash attention backward with the inverse RoPE fused into dQ / dK");
  m.def("ln_fwd", &ln_fwd, "LayerNorm/RMSNorm forward (+fused residual add, + dropout on x)", pybind11::arg("x"),
        pybind11::arg("residual"), pybind11::arg("weight"), pybind11::arg("bias"), pybind11::arg("eps"),
        pybind11::arg("rms"), pybind11::arg("drop_p") = 0.0, pybind11::arg("rng") = pybind11::none());
  m.def("ln_set_waves", [](int64_t w) { hyp::ln_set_waves((int)w); },
        "LayerNorm forward / backward grid: target wave count (A/B; 0 = defaults)");
  m.def("ln_bwd", &ln_bwd, "LayerNorm/RMSNorm backward (+ the dropped input's gradient)", pybind11::arg("dy"),
        pybind11::arg("xin"), pybind11::arg("weight"), pybind11::arg("mean"), pybind11::arg("rstd"),
        pybind11::arg("dres"), pybind11::arg("need_dw"), pybind11::arg("need_db"), pybind11::arg("rms"),
        pybind11::arg("drop_p") = 0.0, pybind11::arg("rng") = pybind11::none(),
        pybind11::arg("branch_sum") = false, pybind11::arg("bsum_dtype") = -1);
}

}  // namespace hypbind
