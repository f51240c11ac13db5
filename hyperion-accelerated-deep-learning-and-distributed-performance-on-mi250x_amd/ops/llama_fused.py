"""One fused autograd node per Llama decoder layer for the frozen-base (LoRA) fine-tune.

Reference: ``train_llama_fsdp(lora=True)`` — HF ``LlamaDecoderLayer`` with PEFT LoRA r16 on
q/k/v/o over a frozen bf16 Llama-2-7B, batch 1 x 128 tokens (``02_development/distributed_utils.py:
463-476, 506-524``; SURVEY C26, §2.4 "GEMM" / "LoRA" / "RMSNorm / RoPE / SwiGLU", §2.5 Llama row).

At 128 tokens the step is the time to stream the frozen weights (13 GB forward + 13 GB data
gradient).  The layer therefore runs as weight-streaming GEMMs (``csrc/kernels/wstream.hip``: x
resident in LDS, W streamed to VGPRs, fp32 fragment-order slabs) with everything else folded into
the slab epilogues or the small LoRA kernels (``csrc/kernels/lora_fused.hip``):

forward  RMSNorm(+residual)  ->  t = drop(h) [A_q A_k A_v]ᵀ (one launch)  ->  h [W_q; W_k; W_v]ᵀ
         (ONE GEMM over the concatenated frozen weight)  ->  epilogue: + c' t Bᵀ per segment, RoPE
         on q / k  ->  flash attention on the packed [B, S, 3, H, D] buffer  ->  O projection with
         its LoRA term  ->  RMSNorm(+residual)  ->  h2 [W_gate; W_up]ᵀ (ONE GEMM) with the SwiGLU
         epilogue  ->  down projection.
backward the same GEMMs as NN products over the SAME frozen weights (no transposed copies, no
         weight-gradient buffers), the SwiGLU backward in the down-dgrad epilogue, the LoRA data
         gradient ``keep ∘ (du' A)`` of q, k and v summed inside ONE epilogue (no autograd adds),
         dA / dB in two small launches per projection group.

Dropout on the LoRA input (p = 0.05, PEFT's ``lora_dropout``) uses a hash mask regenerated from
one graph-safe rng record per projection group — never stored.  ``c' = scaling / (1 - p)``.

The fused node is used when the layer's base weights are frozen, the LoRA adapters (if any) sit on
exactly q/k/v/o, there is no grouped-query attention, head_dim is 128 and the token count is small
(<= ``HYPERION_WS_MAX_M``, default 512).  ``q/k/v`` (and ``gate/up``) must be adjacent in memory —
true inside Hyperion's FSDP flat buffers; :func:`fuse_llama_weights` re-homes a plain model's
frozen weights into per-layer concatenated buffers (state-dict keys and values unchanged).
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from . import _native
from .rope import rope_table

WS_MAX_M = int(os.environ.get("HYPERION_WS_MAX_M", "512"))
RANK_SPLITS = 4  # slices of the rank-r split-partial stacks (t: k-splits of lora_down, du: n-splits)
# rank-r LoRA kernels on a side stream, concurrent with the weight-streaming GEMM that reads the
# same activation (lora_down beside the projection, lora_bwd_t beside its data gradient) and with
# the rest of the layer's backward (lora_bwd_a: its dA is only read by the optimizer) — 192
# latency-bound ~7 us launches per Llama-2-7B step that otherwise serialise with the weight
# stream.  Fork / join are stream-event edges, so a captured step keeps the overlap.  Measured
# SLOWER (graphed Llama-2-7B LoRA step 16.5-16.7 vs 14.9 ms, scripts/gpu_r05s.sh): the rank-r
# workgroups take CU slots from the weight stream and every join is a stream-event wait — opt-in.
LORA_STREAM = os.environ.get("HYPERION_LORA_STREAM", "0") == "1"


class _Side:
    """Fork work onto the LoRA side stream and join it back (no-op when disabled / on CPU)."""

    def __init__(self, dev: torch.device):
        self.on = LORA_STREAM and dev.type == "cuda"
        if self.on:
            from .streams import side_stream

            self.main = torch.cuda.current_stream(dev)
            self.side = side_stream(dev)
        self.pending = False

    def run(self, fn) -> None:
        if not self.on:
            fn()
            return
        self.side.wait_stream(self.main)  # inputs produced so far on the main stream
        with torch.cuda.stream(self.side):
            fn()
        self.pending = True

    def join(self) -> None:
        if self.on and self.pending:
            self.main.wait_stream(self.side)
            self.pending = False
DEBUG: Optional[dict] = None  # tests / scripts: set to a dict to capture the backward intermediates


def _summed(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """A rank-r split-partial stack [S, M, W] as the [M, W] matrix it stands for."""
    return t.sum(0) if t is not None and t.dim() == 3 else t


def _adjacent(ws: List[torch.Tensor]) -> bool:
    """The weights are consecutive row blocks of one contiguous buffer."""
    if not all(w.is_contiguous() for w in ws):
        return False
    for a, b in zip(ws[:-1], ws[1:]):
        if a.untyped_storage().data_ptr() != b.untyped_storage().data_ptr():
            return False
        if a.data_ptr() + a.numel() * a.element_size() != b.data_ptr():
            return False
    return True


def _cat_view(ws: List[torch.Tensor]) -> torch.Tensor:
    """[sum rows, cols] view over adjacent row blocks."""
    rows = sum(w.shape[0] for w in ws)
    base = ws[0]
    return torch.as_strided(base, (rows, base.shape[1]), (base.shape[1], 1))


def _base_weight(mod: nn.Module) -> torch.Tensor:
    return mod.base_layer.weight if hasattr(mod, "base_layer") else mod.weight


def _lora_parts(mod: nn.Module):
    if not hasattr(mod, "lora_A"):
        return None
    a = mod.adapter
    return mod.lora_A[a].weight, mod.lora_B[a].weight, float(mod.scaling[a]), float(mod.p)


def _fuse_layer(m: nn.Module) -> int:
    at, mlp = m.self_attn, m.mlp
    n = 0
    for mods in ((at.q_proj, at.k_proj, at.v_proj), (mlp.gate_proj, mlp.up_proj)):
        ws = [_base_weight(x) for x in mods]
        if any(w.requires_grad for w in ws) or _adjacent(ws):
            continue
        with torch.no_grad():
            buf = torch.cat([w.detach() for w in ws], 0)
            o = 0
            for w in ws:
                w.data = buf[o:o + w.shape[0]]
                o += w.shape[0]
        n += 1
    return n


def fuse_llama_weights(model: nn.Module) -> int:
    """Re-home every decoder layer's frozen q/k/v and gate/up weights into concatenated buffers
    (``p.data`` becomes a view; Parameter objects, keys and values are unchanged).  Returns the
    number of groups changed.  The fused node also does this lazily on its first eager call;
    Hyperion's FSDP flat buffers already hold them adjacent."""
    return sum(_fuse_layer(m) for m in model.modules() if hasattr(m, "self_attn") and hasattr(m, "mlp"))


class _Spec:
    """Per-call constants of one layer (frozen tensors, config) handed to the autograd node."""

    __slots__ = ("W_qkv", "W_o", "W_gu", "W_d", "w1", "w2", "eps", "nh", "hd", "H", "I", "theta", "lora", "c",
                 "p", "r")


def _ln_w32(layer: nn.Module, name: str) -> torch.Tensor:
    """fp32 copy of a frozen RMSNorm weight, cached per (storage, version)."""
    w = getattr(layer, name).weight
    if w.dtype == torch.float32:
        return w.detach()
    key = (w.data_ptr(), w._version)
    cache = layer.__dict__.setdefault("_hyp_w32", {})
    hit = cache.get(name)
    if hit is None or hit[0] != key:
        hit = (key, w.detach().float())
        cache[name] = hit
    return hit[1]


def fused_spec(layer: nn.Module, x: torch.Tensor, kpm: Optional[torch.Tensor]) -> Optional[_Spec]:
    """The layer's fused-node constants, or None when the fused node does not apply."""
    if not (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and _native.use_native(x, op="ws")):
        return None
    cfg = layer.self_attn.cfg
    M = x.shape[0] * x.shape[1]
    if (M > WS_MAX_M or cfg.num_key_value_heads != cfg.num_attention_heads or cfg.head_dim != 128
            or cfg.hidden_size % 128 or cfg.intermediate_size % 64):
        return None
    at, mlp = layer.self_attn, layer.mlp
    qkv = [at.q_proj, at.k_proj, at.v_proj]
    ws = [_base_weight(m) for m in qkv + [at.o_proj, mlp.gate_proj, mlp.up_proj, mlp.down_proj]]
    if any(w.requires_grad or w.dtype != x.dtype for w in ws):
        return None
    if (layer.input_layernorm.weight.requires_grad or layer.post_attention_layernorm.weight.requires_grad
            or any(hasattr(m, "lora_A") for m in (mlp.gate_proj, mlp.up_proj, mlp.down_proj))):
        return None
    if any(getattr(m, "base_layer", m).bias is not None for m in qkv + [at.o_proj]):
        return None
    lp = [_lora_parts(m) for m in qkv + [at.o_proj]]
    if any(p is None for p in lp) and not all(p is None for p in lp):
        return None
    lora = lp[0] is not None
    if lora:
        if len({(p[2], p[3], p[0].shape[0]) for p in lp}) != 1 or any(p[0].dtype != x.dtype or p[1].dtype != x.dtype
                                                                      for p in lp):
            return None
        if lp[0][0].shape[0] > 16:
            return None
    if not (_adjacent(ws[:3]) and _adjacent(ws[4:6])):
        if torch.cuda.is_current_stream_capturing() or not _fuse_layer(layer):
            return None
        ws = [_base_weight(m) for m in qkv + [at.o_proj, mlp.gate_proj, mlp.up_proj, mlp.down_proj]]
        if not (_adjacent(ws[:3]) and _adjacent(ws[4:6])):
            return None
    s = _Spec()
    s.W_qkv, s.W_o, s.W_gu, s.W_d = _cat_view(ws[:3]), ws[3], _cat_view(ws[4:6]), ws[6]
    s.w1, s.w2 = _ln_w32(layer, "input_layernorm"), _ln_w32(layer, "post_attention_layernorm")
    s.eps = layer.input_layernorm.variance_epsilon
    s.nh, s.hd, s.H, s.I = cfg.num_attention_heads, cfg.head_dim, cfg.hidden_size, cfg.intermediate_size
    s.theta = float(cfg.rope_theta)
    s.lora = lora
    if lora:
        _, _, scaling, p = lp[0]
        s.p = p if layer.training else 0.0
        s.c = scaling / (1.0 - s.p)
        s.r = lp[0][0].shape[0]
    else:
        s.p, s.c, s.r = 0.0, 0.0, 0
    return s


# Per-shape GEMM plan: ("ws", mf, kr, G, nf) — the weight-streaming kernel with that plan (0 =
# automatic) — or ("vendor",) — hipBLASLt, its bf16 output then run through the same epilogue kernel
# (``ws_epilogue(yin=...)``).  Filled from cold-weight sweeps (scripts/ws_bench.py,
# profiles/r03/ws_bench.json); ``HYPERION_WS_PLAN=ws|vendor`` forces one side for A/B runs.
_PLAN_OVERRIDE = os.environ.get("HYPERION_WS_PLAN", "")
# split-K partial slabs in bf16 (default): the slabs of the data-gradient GEMMs (24-43 slices of 512
# reduction terms at 128 tokens) were a third of the HBM traffic of those GEMMs and all of their
# epilogues' reads; each slab is one rounding of a fp32 partial, the slabs are summed in fp32.
# HYPERION_WS_SLAB=fp32 keeps fp32 slabs (A/B runs)
SLAB16 = os.environ.get("HYPERION_WS_SLAB", "bf16") != "fp32"
# (nn, output width, reduction length) -> plan; measured at 128 tokens (scripts/ws_bench.py, cold
# weights, GEMM + epilogue): hipBLASLt streams the wide forward projections (q/k/v 12288 x 4096:
# 31.9 us, gate/up 22016 x 4096: 46.7 us — no split-K, activations re-read from L2) faster than
# the slab kernel (43.5 / 74.1 us); every data gradient (hipBLASLt NN 38.6-114 us) and the
# 4096-wide forwards stay on the weight-streaming kernel.
PLANS = {
    (False, 12288, 4096): ("vendor",),
    (False, 22016, 4096): ("vendor",),
    (False, 4096, 11008): ("ws", 8, 512, 11, 1),
}


# cold-weight sweep with bf16 slabs (scripts/ws_bench.py, profiles/r03/ws_bench_bf16_slabs.json):
# GEMM-only best plans — q/k/v forward now streams faster than hipBLASLt (28.1 vs 32.3 us)
PLANS_BF16 = {
    (False, 12288, 4096): ("ws", 8, 512, 32, 1),
    (False, 4096, 4096): ("ws", 8, 512, 32, 1),
    (True, 4096, 4096): ("ws", 8, 256, 16, 4),
    (True, 4096, 22016): ("ws", 8, 384, 4, 4),
    (True, 11008, 4096): ("ws", 8, 384, 23, 4),
}
if SLAB16 and os.environ.get("HYPERION_WS_PLANS", "bf16") == "bf16":
    PLANS = {**PLANS, **PLANS_BF16}


def plan_for(nn_: bool, M: int, N: int, K: int) -> tuple:
    if _PLAN_OVERRIDE == "vendor":
        return ("vendor",)
    if _PLAN_OVERRIDE == "ws":
        return ("ws", 0, 0, 0, 0)
    return PLANS.get((nn_, N, K), ("ws", 0, 0, 0, 0))


class _Proj:
    """One projection's GEMM result: fp32 slabs of the weight-streaming kernel, or a dense vendor output."""

    __slots__ = ("part", "S", "MFt", "y")

    def __init__(self, C, x, w, nn_: bool = False):
        M, K = x.shape
        N = w.shape[1] if nn_ else w.shape[0]
        p = plan_for(nn_, M, N, K)
        self.part = self.y = None
        self.S = self.MFt = 0
        if p[0] == "vendor":
            self.y = x @ w if nn_ else x @ w.t()
        else:
            self.part, self.S, self.MFt = C.ws_gemm_part(x, w, nn=nn_, mf=p[1], kr=p[2], G=p[3], nf=p[4],
                                                         slab16=SLAB16)

    def epi(self, C, M, N, epi, out, **kw):
        C.ws_epilogue(self.part, self.S, self.MFt, M, N, epi, out, yin=self.y, **kw)


class _LlamaLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, delta, stream, kpm, spec: _Spec, Aq, Bq, Ak, Bk, Av, Bv, Ao, Bo):
        C = _native.native()
        Bsz, S, H = stream.shape
        M = Bsz * S
        dt = stream.dtype
        dev = stream.device
        xs = stream.reshape(M, H).contiguous()
        if delta is None:
            h, _, _, rstd1 = C.ln_fwd(xs, None, spec.w1, None, spec.eps, True)
            s = xs
        else:
            h, s, _, rstd1 = C.ln_fwd(delta.reshape(M, H).contiguous(), xs, spec.w1, None, spec.eps, True)
        lora = spec.lora
        rq = ro = None
        t_qkv = t_o = du_bufs = t_all = None
        if lora:
            if spec.p > 0:
                rq, ro = _native.rng_state(dev), _native.rng_state(dev)
            # t (k-split) and du (n-split) as fp32 split-partial stacks [S, M, 4 r] — q/k/v columns
            # then o — written slice by slice by lora_down / lora_bwd_t and summed by every consumer:
            # no atomics, no fill kernels, and the rank-r work spreads over ~100-200 workgroups
            t_all = torch.empty(RANK_SPLITS, M, 4 * spec.r, device=dev, dtype=torch.float32)
            t_qkv = t_all[:, :, :3 * spec.r]
            du_bufs = torch.empty(RANK_SPLITS, M, 4 * spec.r, device=dev, dtype=torch.float32)
        side = _Side(dev)
        if lora:
            side.run(lambda: C.lora_down(h, [Aq, Ak, Av], t_qkv, rq, spec.p))
        pj = _Proj(C, h, spec.W_qkv)
        qkv = torch.empty(M, 3 * H, device=dev, dtype=dt)
        side.join()
        pj.epi(C, M, 3 * H, 1, qkv, t=t_qkv, lw=[Bq, Bk, Bv] if lora else [], segw=H,
                      lscale=spec.c, rope_segs=2, seq=S, theta=spec.theta)
        q5 = qkv.view(Bsz, S, 3, spec.nh, spec.hd)
        q, k, v = q5[:, :, 0], q5[:, :, 1], q5[:, :, 2]
        scale = 1.0 / math.sqrt(spec.hd)
        o, lse = C.attn_fwd(q, k, v, True, scale, 0.0, None, kpm, True)
        o2 = o.view(M, H)
        if lora:
            t_o = t_all[:, :, 3 * spec.r:]
            side.run(lambda: C.lora_down(o2, [Ao], t_o, ro, spec.p))
        pj = _Proj(C, o2, spec.W_o)
        a = torch.empty(M, H, device=dev, dtype=dt)
        side.join()
        pj.epi(C, M, H, 1, a, t=t_o, lw=[Bo] if lora else [], segw=H, lscale=spec.c)
        h2, s2, _, rstd2 = C.ln_fwd(a, s, spec.w2, None, spec.eps, True)
        pj = _Proj(C, h2, spec.W_gu)
        gu = torch.empty(M, 2 * spec.I, device=dev, dtype=dt)
        hh = torch.empty(M, spec.I, device=dev, dtype=dt)
        pj.epi(C, M, 2 * spec.I, 2, gu, out2=hh)
        pj = _Proj(C, hh, spec.W_d)
        d = torch.empty(M, H, device=dev, dtype=dt)
        pj.epi(C, M, H, 0, d)
        ctx.spec = spec
        ctx.cfg = (Bsz, S, delta is not None, scale, rq, ro)
        ctx.save_for_backward(h, s, rstd1, qkv, o, lse, s2, rstd2, gu, kpm, t_qkv, t_o, du_bufs if lora else None, Aq, Bq,
                              Ak, Bk, Av, Bv, Ao, Bo)
        return d.view(Bsz, S, H), s2.view(Bsz, S, H)

    @staticmethod
    def backward(ctx, dd, ds2):
        C = _native.native()
        spec: _Spec = ctx.spec
        Bsz, S, has_delta, scale, rq, ro = ctx.cfg
        (h, s, rstd1, qkv, o, lse, s2, rstd2, gu, kpm, t_qkv, t_o, du_bufs, Aq, Bq, Ak, Bk, Av, Bv, Ao,
         Bo) = ctx.saved_tensors
        H, I = spec.H, spec.I
        M = Bsz * S
        dt, dev = h.dtype, h.device
        lora = spec.lora
        dd2 = dd.reshape(M, H).to(dt).contiguous() if dd is not None else torch.zeros(M, H, device=dev, dtype=dt)
        ds2c = ds2.reshape(M, H).to(dt).contiguous() if ds2 is not None else None
        # down projection: dhh = dd W_d, SwiGLU backward in the epilogue -> dgu [M, 2I]
        pj = _Proj(C, dd2, spec.W_d, True)
        dgu = torch.empty(M, 2 * I, device=dev, dtype=dt)
        pj.epi(C, M, I, 3, dgu, aux=gu)
        # gate/up: dh2 = dgu [W_gate; W_up]
        pj = _Proj(C, dgu, spec.W_gu, True)
        dh2 = torch.empty(M, H, device=dev, dtype=dt)
        pj.epi(C, M, H, 0, dh2, nn=True)
        dsum2 = C.ln_bwd(dh2, s2, spec.w2, rstd2, rstd2, ds2c, False, False, True)[0]  # grad of s2 = a + s
        # O projection (+ LoRA)
        grads = [None] * 8
        du_o = None
        side = _Side(dev)
        if lora:
            du_o = du_bufs[:, :, 3 * spec.r:]
            dAo, dBo = torch.empty_like(Ao), torch.empty_like(Bo)
            side.run(lambda: C.lora_bwd_t(dsum2, H, [Bo], [dBo], t_o, du_o, spec.c))
        pj = _Proj(C, dsum2, spec.W_o, True)
        do = torch.empty(M, H, device=dev, dtype=dt)
        if lora:
            side.join()
            pj.epi(C, M, H, 4, do, t=du_o, lw=[Ao], rng=ro, p_drop=spec.p)
            side.run(lambda: C.lora_bwd_a(o.view(M, H), [dAo], du_o, ro, spec.p))  # joined at the end
            grads[6], grads[7] = dAo, dBo
        else:
            pj.epi(C, M, H, 0, do, nn=True)
        # attention backward straight into the packed gradient, RoPE backward in place
        q5 = qkv.view(Bsz, S, 3, spec.nh, spec.hd)
        dqkv = torch.empty(M, 3 * H, device=dev, dtype=dt)
        d5 = dqkv.view(Bsz, S, 3, spec.nh, spec.hd)
        dq, dk, dv = d5[:, :, 0], d5[:, :, 1], d5[:, :, 2]
        if spec.hd == 128:  # inverse RoPE fused into the attention backward's dQ / dK stores
            C.attn_bwd_rope(do.view(Bsz, S, spec.nh, spec.hd), q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], o, lse, True,
                            scale, kpm, dq, dk, dv, rope_table(S, spec.hd, spec.theta, dev))
        else:
            C.attn_bwd(do.view(Bsz, S, spec.nh, spec.hd), q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], o, lse, True, scale,
                       0.0, None, kpm, dq, dk, dv)
            C.rope_(dq, dk, None, spec.theta, True)
        # q/k/v: dh = dqkv [W_q; W_k; W_v] + Σ_p keep_p ∘ (du'_p A_p)
        du_qkv = None
        if lora:
            du_qkv = du_bufs[:, :, :3 * spec.r]
            dA = [torch.empty_like(Aq), torch.empty_like(Ak), torch.empty_like(Av)]
            dB = [torch.empty_like(Bq), torch.empty_like(Bk), torch.empty_like(Bv)]
            side.run(lambda: C.lora_bwd_t(dqkv, H, [Bq, Bk, Bv], dB, t_qkv, du_qkv, spec.c))
        pj = _Proj(C, dqkv, spec.W_qkv, True)
        dh = torch.empty(M, H, device=dev, dtype=dt)
        if lora:
            side.join()
            pj.epi(C, M, H, 4, dh, t=du_qkv, lw=[Aq, Ak, Av], rng=rq, p_drop=spec.p)
            side.run(lambda: C.lora_bwd_a(h, dA, du_qkv, rq, spec.p))
            grads[0], grads[1], grads[2], grads[3], grads[4], grads[5] = dA[0], dB[0], dA[1], dB[1], dA[2], dB[2]
        else:
            pj.epi(C, M, H, 0, dh, nn=True)
        dsum1 = C.ln_bwd(dh, s, spec.w1, rstd1, rstd1, dsum2, False, False, True)[0]
        side.join()  # dA of q/k/v and o: the gradients returned below are read on the main stream
        if DEBUG is not None:
            DEBUG.update(dgu=dgu, dh2=dh2, dsum2=dsum2, do=do, dqkv=dqkv, dh=dh, dsum1=dsum1, h=h, s=s, qkv=qkv, o=o,
                         s2=s2, gu=gu, dd=dd2, ds2=ds2c, t_qkv=_summed(t_qkv), t_o=_summed(t_o), du_o=_summed(du_o),
                         du_qkv=_summed(du_qkv))
        d_in = dsum1.view(Bsz, S, H)
        return (d_in if has_delta else None, d_in, None, None, *grads)


def llama_layer_fused(layer: nn.Module, delta: Optional[torch.Tensor], stream: torch.Tensor,
                      kpm: Optional[torch.Tensor]) -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
    """Run ``layer`` (a LlamaDecoderLayer, residual-stream form) as one fused node, or return None."""
    spec = fused_spec(layer, stream, kpm)
    if spec is None:
        return None
    at = layer.self_attn
    if spec.lora:
        lp = [_lora_parts(m) for m in (at.q_proj, at.k_proj, at.v_proj, at.o_proj)]
        ab = [t for p in lp for t in (p[0], p[1])]
    else:
        dummy = stream.new_empty(0)
        ab = [dummy] * 8
    k8 = kpm.to(torch.uint8) if kpm is not None else None
    return _LlamaLayerFn.apply(delta, stream, k8, spec, *ab)
