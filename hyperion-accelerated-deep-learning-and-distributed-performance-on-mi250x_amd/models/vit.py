"""ViT-B/16 (torchvision-key compatible) and the reference's fallback CNN.

Reference: ``create_vit_model()`` tried torchvision ``vit_b_16(pretrained=False)`` and, because
torchvision lacked it on that install, fell back to a 5-layer CNN — the "Vision Transformer"
row of the README (5.44 ms, batch 32) is that CNN (``Phase 1/baseline_performance.ipynb:207-236``,
fallback proof :28-29).  Hyperion provides both, so one comparison is
like-for-like (``fallback_cnn``) and the other is the real model (``vit_b_16``).

ViT design for MI355X: pre-norm blocks whose residual adds are fused into the next LayerNorm
(``layer_norm(..., residual=r, return_sum=True)`` returns both ``LN(x + r)`` and ``x + r`` in one
pass), packed-QKV flash attention on ``[B, 197, 3, 12, 64]`` without permutes, GELU in the FC1
GEMM epilogue.  ``use_checkpoint=True`` recomputes each encoder block in backward (the
BASELINE.json "ViT-Base bf16 + activation checkpointing" config); ``use_checkpoint="selective"``
keeps the GEMM outputs and rebuilds only the LayerNorm / GELU outputs (``ops/recompute.py``).  State-dict keys equal
torchvision's (``conv_proj``, ``class_token``, ``encoder.pos_embedding``,
``encoder.layers.encoder_layer_N.{ln_1,self_attention,ln_2,mlp.0,mlp.3}``, ``encoder.ln``,
``heads.head``).
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Optional, Tuple

import torch
import torch.nn as nn

from ..ops.pool import AdaptiveAvgPool2d, MaxPool2d
from torch.utils.checkpoint import checkpoint

from ..ops import recompute as _rc
from ..ops.conv_f32 import Conv2d
from ..ops.dropout import Dropout
from ..ops.layernorm import LayerNorm, bias_grad_link, layer_norm
from ..ops.linear import Linear
from ..ops.linear_act import LinearAct
from .transformer import MultiheadSelfAttention, _ffn_up


class MLPBlock(nn.Sequential):
    """torchvision ``MLPBlock`` layout: ``0`` Linear, ``1`` GELU, ``2`` Dropout, ``3`` Linear, ``4`` Dropout."""

    def __init__(self, dim: int, hidden: int, dropout: float = 0.0):
        # [0] applies the GELU itself (bias + GELU with the GEMM); [1] stays for the torchvision layout
        super().__init__(LinearAct(dim, hidden, activation="gelu"), nn.GELU(), Dropout(dropout),
                         Linear(hidden, dim), Dropout(dropout))
        for m in (self[0], self[3]):
            nn.init.xavier_uniform_(m.weight)
            nn.init.normal_(m.bias, std=1e-6)

    def forward(self, x: torch.Tensor, blink=None) -> torch.Tensor:  # type: ignore[override]
        return self[4](self[3](self[2](self[0](x)), blink=blink))


class EncoderBlock(nn.Module):
    def __init__(self, num_heads: int, hidden_dim: int, mlp_dim: int, dropout: float = 0.0,
                 attention_dropout: float = 0.0):
        super().__init__()
        self.num_heads = num_heads
        self.ln_1 = LayerNorm(hidden_dim, eps=1e-6)
        self.self_attention = MultiheadSelfAttention(hidden_dim, num_heads, dropout=attention_dropout)
        self.dropout = Dropout(dropout)
        self.ln_2 = LayerNorm(hidden_dim, eps=1e-6)
        self.mlp = MLPBlock(hidden_dim, mlp_dim, dropout)

    def forward(self, delta: Optional[torch.Tensor], stream: torch.Tensor, blink_in=None,
                blink_out=None) -> Tuple[torch.Tensor, torch.Tensor]:  # type: ignore[override]
        """One block on the residual stream.

        Input ``stream + delta`` is the block input (``delta`` = previous block's MLP output, not yet
        added).  Returns ``(mlp_out, new_stream)`` with ``new_stream + mlp_out`` = block output.
        ``blink_in`` / ``blink_out``: BiasGradLinks of the previous / this block's fc2 (its bias
        gradient is the column sum the next LayerNorm backward takes of its input gradient); the
        attention out_proj's bias gradient comes from ln_2's backward the same way.
        """
        if delta is None:
            h, s = self.ln_1(stream), stream
        else:
            h, s = layer_norm(delta, self.ln_1.weight, self.ln_1.bias, self.ln_1.eps, residual=stream,
                              return_sum=True, blink=blink_in)
        bl = bias_grad_link()
        a = self.dropout(self.self_attention(h, blink=bl))
        h2, s2 = layer_norm(a, self.ln_2.weight, self.ln_2.bias, self.ln_2.eps, residual=s, return_sum=True, blink=bl)
        return self.mlp(h2, blink=blink_out), s2

    def block(self, x: torch.Tensor) -> torch.Tensor:
        """Plain form: x -> block output."""
        d, s = self(None, x)
        return s + d


class Encoder(nn.Module):
    def __init__(self, seq_length: int, num_layers: int, num_heads: int, hidden_dim: int, mlp_dim: int,
                 dropout: float = 0.0, attention_dropout: float = 0.0, use_checkpoint: bool = False):
        super().__init__()
        self.pos_embedding = nn.Parameter(torch.empty(1, seq_length, hidden_dim).normal_(std=0.02))
        self.dropout = Dropout(dropout)
        self.layers = nn.ModuleDict(
            OrderedDict(
                (f"encoder_layer_{i}", EncoderBlock(num_heads, hidden_dim, mlp_dim, dropout, attention_dropout))
                for i in range(num_layers)
            )
        )
        self.ln = LayerNorm(hidden_dim, eps=1e-6)
        self.use_checkpoint = use_checkpoint

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.use_checkpoint == "selective":
            # keep the GEMM outputs, rebuild LayerNorm / GELU outputs in backward (ops/recompute.py)
            with _rc.selective(self.training):
                return self._forward(x, False)
        return self._forward(x, bool(self.use_checkpoint) and self.training and torch.is_grad_enabled())

    def _forward(self, x: torch.Tensor, ckpt: bool) -> torch.Tensor:
        s = self.dropout(x + self.pos_embedding.to(x.dtype))
        d: Optional[torch.Tensor] = None
        for blk in self.layers.values():
            if ckpt:
                if d is None:
                    d, s = checkpoint(blk, None, s, use_reentrant=False)
                else:
                    d, s = checkpoint(blk, d, s, use_reentrant=False)
            else:
                bl_prev = bl if d is not None else None
                bl = bias_grad_link()
                d, s = blk(d, s, blink_in=bl_prev, blink_out=bl)
        if d is None:
            return self.ln(s)
        return self.ln(d, residual=s, blink=None if ckpt else bl)


class VisionTransformer(nn.Module):
    def __init__(self, image_size: int = 224, patch_size: int = 16, num_layers: int = 12, num_heads: int = 12,
                 hidden_dim: int = 768, mlp_dim: int = 3072, dropout: float = 0.0, attention_dropout: float = 0.0,
                 num_classes: int = 1000, use_checkpoint: bool = False):
        super().__init__()
        if image_size % patch_size:
            raise ValueError("image size must be divisible by the patch size")
        self.image_size = image_size
        self.patch_size = patch_size
        self.hidden_dim = hidden_dim
        self.conv_proj = Conv2d(3, hidden_dim, kernel_size=patch_size, stride=patch_size)
        seq_length = (image_size // patch_size) ** 2 + 1
        self.class_token = nn.Parameter(torch.zeros(1, 1, hidden_dim))
        self.encoder = Encoder(seq_length, num_layers, num_heads, hidden_dim, mlp_dim, dropout, attention_dropout,
                               use_checkpoint)
        self.seq_length = seq_length
        self.heads = nn.Sequential(OrderedDict(head=nn.Linear(hidden_dim, num_classes)))
        fan_in = 3 * patch_size * patch_size
        nn.init.trunc_normal_(self.conv_proj.weight, std=math.sqrt(1 / fan_in))
        nn.init.zeros_(self.conv_proj.bias)
        nn.init.zeros_(self.heads.head.weight)
        nn.init.zeros_(self.heads.head.bias)

    @property
    def use_checkpoint(self) -> bool:
        return self.encoder.use_checkpoint

    @use_checkpoint.setter
    def use_checkpoint(self, v) -> None:
        """True: every block recomputed in backward; "selective": GEMM outputs kept, LayerNorm /
        GELU outputs rebuilt (ops/recompute.py); False: nothing recomputed."""
        self.encoder.use_checkpoint = v if v == "selective" else bool(v)

    def _process_input(self, x: torch.Tensor) -> torch.Tensor:
        """Patch embedding.  A p x p / stride-p convolution over non-overlapping patches IS a GEMM:
        patches [n·(h/p)·(w/p), c·p·p] (one permute copy, in the conv weight's (c, kh, kw) order)
        times the flattened weight — the tokens come out already as [n, h/p·w/p, hidden], and the
        backward is a plain weight-gradient GEMM.  (MIOpen has no fast bf16 NHWC solver for the
        3-channel 16x16/16 conv: it ran its naive reference kernels, 11 ms forward + 7 ms wrw per
        ViT-B/16 step on MI355X, profiles/r02/vit_b16_kernels.)"""
        n, c, h, w = x.shape
        if h != self.image_size or w != self.image_size:
            raise ValueError(f"expected {self.image_size}x{self.image_size} input, got {h}x{w}")
        p = self.patch_size
        wt = self.conv_proj.weight
        x = x.to(wt.dtype) if not torch.is_autocast_enabled(x.device.type) else x
        patches = (x.reshape(n, c, h // p, p, w // p, p).permute(0, 2, 4, 1, 3, 5)
                   .reshape(n * (h // p) * (w // p), c * p * p))
        tok = torch.nn.functional.linear(patches, wt.reshape(wt.shape[0], -1), self.conv_proj.bias)
        return tok.reshape(n, (h // p) * (w // p), self.hidden_dim)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self._process_input(x)
        cls = self.class_token.to(x.dtype).expand(x.shape[0], -1, -1)
        x = torch.cat([cls, x], dim=1)
        x = self.encoder(x)
        return self.heads(x[:, 0])


def vit_b_16(num_classes: int = 1000, image_size: int = 224, use_checkpoint: bool = False, **kw) -> VisionTransformer:
    """ViT-B/16: 86.6M parameters at 1000 classes."""
    return VisionTransformer(image_size, 16, 12, 12, 768, 3072, num_classes=num_classes,
                             use_checkpoint=use_checkpoint, **kw)


def vit_tiny(num_classes: int = 10, image_size: int = 32, patch_size: int = 4, **kw) -> VisionTransformer:
    """Small ViT for CPU tests."""
    return VisionTransformer(image_size, patch_size, 2, 4, 64, 128, num_classes=num_classes, **kw)


def fallback_cnn(num_classes: int = 1000) -> nn.Sequential:
    """The CNN the reference actually benchmarked as "ViT" (212,328 params; keys 0/3/7)."""
    return nn.Sequential(
        Conv2d(3, 64, kernel_size=7, stride=2, padding=3),
        nn.ReLU(inplace=True),
        MaxPool2d(kernel_size=3, stride=2, padding=1),
        Conv2d(64, 128, kernel_size=3, padding=1),
        nn.ReLU(inplace=True),
        MaxPool2d(kernel_size=3, stride=2, padding=1),
        AdaptiveAvgPool2d((1, 1)),
        nn.Flatten(),
        nn.Linear(128, num_classes),
    )


def create_vit_model(real: bool = False) -> nn.Module:
    """Reference factory (``baseline_performance.ipynb:207``).

    ``real=False`` (default) reproduces what the reference measured — the fallback CNN;
    ``real=True`` returns ViT-B/16.
    """
    return vit_b_16() if real else fallback_cnn()
