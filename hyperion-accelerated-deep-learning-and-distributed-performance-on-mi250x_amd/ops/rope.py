"""Rotary position embeddings (HF Llama ``rotate_half`` convention) on gfx950.

Reference: HF ``LlamaRotaryEmbedding`` + ``apply_rotary_pos_emb`` inside ``train_llama_fsdp``'s
model (``02_development/distributed_utils.py:465-487``; SURVEY §2.4 "RMSNorm / RoPE / SwiGLU").
One HIP kernel (``csrc/kernels/rope_swiglu.hip``) rotates q and k together, computing the angles
in fp32 on the fly (no cos/sin cache tensors); backward is the inverse rotation.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

from . import _native


def rope_reference(q: torch.Tensor, k: torch.Tensor, positions: Optional[torch.Tensor], theta: float = 10000.0):
    """PyTorch oracle on ``[B, S, H, D]`` tensors (fp32 angles, like the kernel)."""
    B, S, _, D = q.shape
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, device=q.device, dtype=torch.float32) / D))
    pos = positions.float() if positions is not None else torch.arange(S, device=q.device, dtype=torch.float32)[None].expand(B, S)
    ang = pos[..., None] * inv  # [B, S, D/2]
    cos, sin = torch.cos(ang)[:, :, None, :], torch.sin(ang)[:, :, None, :]

    def rot(x):
        xf = x.float()
        x1, x2 = xf[..., : D // 2], xf[..., D // 2 :]
        return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)

    return rot(q), rot(k)


_TABLES: dict = {}


def rope_table(S: int, D: int, theta: float, device) -> torch.Tensor:
    """fp32 [S, D/2, 2] (cos, sin) of position x inv_freq(i), inv_freq = theta^(-2i/D) computed as the
    kernels do (exp2 of -(2i/D) log2 theta); cached per (S, D, theta, device) — built eagerly before
    a hipGraph capture reads it (the fused attention backward's inverse RoPE)."""
    key = (int(S), int(D), float(theta), str(device))
    t = _TABLES.get(key)
    if t is None:
        i = torch.arange(D // 2, device=device, dtype=torch.float32)
        inv = torch.exp2(-(2.0 * i / D) * math.log2(theta))
        ang = torch.arange(S, device=device, dtype=torch.float32)[:, None] * inv[None, :]
        t = torch.stack([torch.cos(ang), torch.sin(ang)], dim=-1).contiguous()
        _TABLES[key] = t
    return t


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, positions, theta):
        qo, ko = _native.native().rope(q, k, positions, float(theta), False)
        ctx.save_for_backward(positions if positions is not None else torch.empty(0))
        ctx.has_pos = positions is not None
        ctx.theta = theta
        ctx.shapes = (q.shape, k.shape)
        return qo, ko

    @staticmethod
    def backward(ctx, dq, dk):
        (pos,) = ctx.saved_tensors
        if dq is None or dk is None:
            ref = dk if dq is None else dq
            shape_q, shape_k = ctx.shapes
            dq = dq if dq is not None else torch.zeros(shape_q, dtype=ref.dtype, device=ref.device)
            dk = dk if dk is not None else torch.zeros(shape_k, dtype=ref.dtype, device=ref.device)
        dqi, dki = _native.native().rope(dq.contiguous(), dk.contiguous(), pos if ctx.has_pos else None,
                                         float(ctx.theta), True)
        return dqi, dki, None, None


def apply_rope(q: torch.Tensor, k: torch.Tensor, positions: Optional[torch.Tensor] = None,
               theta: float = 10000.0) -> Tuple[torch.Tensor, torch.Tensor]:
    D = q.shape[-1]
    if (_native.use_native(q, k, op="rope") and q.dtype in _native.DTYPE_CODE and q.dtype == k.dtype and D % 16 == 0
            and q.stride(-1) == 1 and k.stride(-1) == 1):
        return _native.apply_fn(_RopeFn, q, k, positions, theta)
    return rope_reference(q, k, positions, theta)
