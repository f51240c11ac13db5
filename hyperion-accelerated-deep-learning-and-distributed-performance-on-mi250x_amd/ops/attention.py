"""Softmax attention over the gfx950 flash kernels (``csrc/kernels/attention.hip``).

Tensors are ``[B, S, H, D]`` (sequence-major, heads interleaved) — the natural output of a packed
QKV projection, so no permute/contiguous copies sit between the projection GEMM and the kernel.
``attention_packed(qkv)`` takes the ``[B, S, 3, H, D]`` view directly and returns the gradient
of the packed tensor in one buffer (no slice-grad accumulation).

Reference attention: ``nn.MultiheadAttention`` → SDPA math fallback (C14/C15/C5) and HF Llama
SDPA with a causal mask (C26).  Dropout (p=0.1 in nn.TransformerEncoderLayer) is applied to the
attention probabilities inside the kernel with a counter-based hash (seed, b, h, q, k), so the
backward regenerates the same mask.  The seed / offset come from torch's default generator
(``_native.rng_state``): every hipGraph replay draws a fresh mask, as torch's dropout does.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

from . import _native
from . import recompute as _rc

def _rng(t: torch.Tensor, p: float):
    return _native.rng_state(t.device) if p > 0 else None


def _native_ok(*ts: torch.Tensor) -> bool:
    t = ts[0]
    if t.dtype not in (torch.bfloat16, torch.float16) or t.shape[-1] not in (64, 128):
        return False
    for x in ts:
        if x.stride(-1) != 1 or any(s % 8 for s in x.stride()[:-1]) or x.data_ptr() % 16:
            return False
    return True


def attention_reference(q, k, v, causal=False, dropout_p=0.0, key_padding_mask=None, scale=None):
    """PyTorch SDPA on [B, S, H, D] tensors (oracle / CPU path)."""
    qt, kt, vt = (x.transpose(1, 2) for x in (q, k, v))
    mask = None
    if key_padding_mask is not None:
        mask = ~key_padding_mask.bool()[:, None, None, :]
        if causal:
            S = q.shape[1]
            mask = mask & torch.ones(S, S, dtype=torch.bool, device=q.device).tril()
            causal = False
    o = F.scaled_dot_product_attention(qt, kt, vt, attn_mask=mask, dropout_p=dropout_p, is_causal=causal, scale=scale)
    return o.transpose(1, 2)


def _recipe_o(o, q, k, v, causal, scale, p, seed, kpm) -> None:
    """Selective recompute (ops/recompute.py): the attention output is rebuilt by re-running the
    forward kernel on the saved q / k / v (same dropout seed: bit-identical) for the backward of
    this op and of the output projection, instead of being kept (d_model per token per layer)."""
    if _rc.active():
        _rc.register(o, lambda: _native.native().attn_fwd(q, k, v, causal, scale, p, seed, kpm, True)[0])


class _AttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, dropout_p, kpm, scale):
        seed = _rng(q, dropout_p)
        o, lse = _native.native().attn_fwd(q, k, v, causal, scale, dropout_p, seed, kpm, True)
        ctx.save_for_backward(q, k, v, o, lse, kpm)
        ctx.cfg = (causal, dropout_p, seed, scale)
        _recipe_o(o, q, k, v, causal, scale, dropout_p, seed, kpm)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, kpm = ctx.saved_tensors
        causal, p, seed, scale = ctx.cfg
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _native.native().attn_bwd(do, q, k, v, o, lse, causal, scale, p, seed, kpm, dq, dk, dv)
        return dq, dk, dv, None, None, None, None


class _AttnPackedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, causal, dropout_p, kpm, scale):
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        seed = _rng(q, dropout_p)
        o, lse = _native.native().attn_fwd(q, k, v, causal, scale, dropout_p, seed, kpm, True)
        ctx.save_for_backward(qkv, o, lse, kpm)
        ctx.cfg = (causal, dropout_p, seed, scale)
        _recipe_o(o, q, k, v, causal, scale, dropout_p, seed, kpm)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, kpm = ctx.saved_tensors
        causal, p, seed, scale = ctx.cfg
        dqkv = torch.empty_like(qkv)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        _native.native().attn_bwd(
            do, q, k, v, o, lse, causal, scale, p, seed, kpm, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2]
        )
        return dqkv, None, None, None, None


def attention(
    q: torch.Tensor,
    k: torch.Tensor,
    v: torch.Tensor,
    causal: bool = False,
    dropout_p: float = 0.0,
    key_padding_mask: Optional[torch.Tensor] = None,
    scale: Optional[float] = None,
) -> torch.Tensor:
    """Self-attention on [B, S, H, D]; ``key_padding_mask`` [B, S] True = ignore that key."""
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else scale
    if _native.use_native(q, op="attn") and q.shape == k.shape == v.shape and _native_ok(q, k, v):
        kpm = key_padding_mask.to(torch.uint8) if key_padding_mask is not None else None
        return _native.apply_fn(_AttnFn, q, k, v, causal, float(dropout_p), kpm, scale)
    return attention_reference(q, k, v, causal, dropout_p, key_padding_mask, scale)


def attention_packed(
    qkv: torch.Tensor,
    causal: bool = False,
    dropout_p: float = 0.0,
    key_padding_mask: Optional[torch.Tensor] = None,
    scale: Optional[float] = None,
) -> torch.Tensor:
    """Self-attention from a packed ``[B, S, 3, H, D]`` projection output; returns [B, S, H, D]."""
    scale = 1.0 / math.sqrt(qkv.shape[-1]) if scale is None else scale
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    if _native.use_native(qkv, op="attn") and _native_ok(q, k, v):
        kpm = key_padding_mask.to(torch.uint8) if key_padding_mask is not None else None
        return _native.apply_fn(_AttnPackedFn, qkv, causal, float(dropout_p), kpm, scale)
    return attention_reference(q, k, v, causal, dropout_p, key_padding_mask, scale)
