"""Transformer encoder blocks with ``nn.TransformerEncoderLayer`` state-dict keys.

Reference users:
* ``SimpleTransformerLM`` (256-d, 2 layers, ReLU, ``batch_first=False``) —
  ``02_development/distributed_utils.py:75-88`` (C14);
* the 768-d LM of the compile bench (GELU, 4 layers) — ``compilation_optimization.py:57-71`` (C15);
* ``CustomTransformer`` (512-d, 6 layers, ``batch_first=True``) —
  ``Phase 1/baseline_performance.ipynb:238-249`` (C5).

All of them use PyTorch's post-norm encoder layer::

    x = norm1(x + dropout1(self_attn(x)))
    x = norm2(x + dropout2(linear2(dropout(act(linear1(x))))))

MI355X design.  Activations are kept batch-major ``[B, S, E]`` inside the stack whatever the
caller's layout (attention is independent per sequence, so ``batch_first=False`` only changes
the view at the boundary — the reference's two ``permute`` copies per forward disappear).  The
packed QKV projection output is viewed as ``[B, S, 3, H, Dh]`` and handed straight to the
flash-attention kernel (``ops.attention.attention_packed``: no split/permute/contiguous), the
residual add AND the residual branch's dropout (``dropout1`` / ``dropout2``) are fused into the
LayerNorm kernel (``ops.layernorm``), and the FFN's bias+activation
rides the GEMM epilogue (``ops.linear_act``: ``torch._addmm_activation`` → hipBLASLt epilogue).
Parameter names match ``nn.TransformerEncoderLayer`` / ``nn.TransformerEncoder`` exactly
(``self_attn.in_proj_weight`` …, ``layers.N.…``) so reference checkpoints load unchanged.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.checkpoint import checkpoint

from ..ops.attention import attention_packed
from ..ops.conv import residual_link
from ..ops.dropout import Dropout
from ..ops.layernorm import LayerNorm, bias_grad_link
from ..ops.linear import Linear, linear
from ..ops.linear_act import LinearAct, linear_act


class MultiheadSelfAttention(nn.Module):
    """Self-attention with ``nn.MultiheadAttention`` parameter names (packed in-projection)."""

    def __init__(self, embed_dim: int, num_heads: int, dropout: float = 0.0, bias: bool = True):
        super().__init__()
        if embed_dim % num_heads:
            raise ValueError("embed_dim must be divisible by num_heads")
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        self.dropout = dropout
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * embed_dim)) if bias else None
        self.out_proj = Linear(embed_dim, embed_dim, bias=bias)
        self._reset_parameters()

    def _reset_parameters(self) -> None:  # same init as nn.MultiheadAttention
        nn.init.xavier_uniform_(self.in_proj_weight)
        if self.in_proj_bias is not None:
            nn.init.zeros_(self.in_proj_bias)
            nn.init.zeros_(self.out_proj.bias)

    def forward(
        self,
        x: torch.Tensor,
        causal: bool = False,
        key_padding_mask: Optional[torch.Tensor] = None,
        link=None,
        blink=None,
    ) -> torch.Tensor:
        B, S, E = x.shape
        qkv = linear(x, self.in_proj_weight, self.in_proj_bias, link=link).view(B, S, 3, self.num_heads, self.head_dim)
        p = self.dropout if self.training else 0.0
        o = attention_packed(qkv, causal=causal, dropout_p=p, key_padding_mask=key_padding_mask)
        return self.out_proj(o.reshape(B, S, E), blink=blink)


def _ffn_up(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], activation: str) -> torch.Tensor:
    """``act(x @ w.T + b)``; bias + ReLU ride the hipBLASLt epilogue on GPU (``ops.linear_act``)."""
    return linear_act(x, w, b, activation)


class TransformerEncoderLayer(nn.Module):
    """Post-norm (default) or pre-norm encoder layer; ``nn.TransformerEncoderLayer`` keys."""

    def __init__(
        self,
        d_model: int,
        nhead: int,
        dim_feedforward: int = 2048,
        dropout: float = 0.1,
        activation: str = "relu",
        layer_norm_eps: float = 1e-5,
        norm_first: bool = False,
        bias: bool = True,
    ):
        super().__init__()
        if activation not in ("relu", "gelu"):
            raise ValueError(f"activation {activation!r}")
        self.self_attn = MultiheadSelfAttention(d_model, nhead, dropout=dropout, bias=bias)
        # modules called as modules (FSDP gathers a unit's shard in its forward pre-hook)
        self.linear1 = LinearAct(d_model, dim_feedforward, bias=bias, activation=activation)
        self.dropout = Dropout(dropout)
        self.linear2 = Linear(dim_feedforward, d_model, bias=bias)
        self.norm_first = norm_first
        self.norm1 = LayerNorm(d_model, eps=layer_norm_eps)
        self.norm2 = LayerNorm(d_model, eps=layer_norm_eps)
        self.dropout1 = Dropout(dropout)
        self.dropout2 = Dropout(dropout)
        self.activation = activation

    def _ff(self, x: torch.Tensor, link=None, blink=None) -> torch.Tensor:
        # the inner dropout rides linear1's epilogue (forward) and its activation backward
        return self.linear2(self.linear1(x, dropout_p=self.dropout.p if self.training else 0.0, link=link),
                            blink=blink)

    def forward(self, x: torch.Tensor, causal: bool = False,
                key_padding_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        if self.norm_first:
            x = x + self.dropout1(self.self_attn(self.norm1(x), causal, key_padding_mask))
            return x + self.dropout2(self._ff(self.norm2(x)))
        # LN(x + dropout(branch)) in one kernel each: the residual branches' dropouts ride the norms
        # (mask regenerated in the LN forward and backward kernels: no dropout launch, no mask tensor)
        # The layer input feeds the QKV GEMM and norm1's residual (then norm1's output feeds linear1 and
        # norm2's residual): each norm's backward parks the residual gradient in a ResidualLink and
        # the GEMM's data gradient adds it in its epilogue — no autograd add of the two gradients
        p1 = self.dropout1.p if self.training else 0.0
        p2 = self.dropout2.p if self.training else 0.0
        # and out_proj's / linear2's bias gradients come from the norm backward's column sums (BiasGradLink)
        link = residual_link(x) if torch.is_grad_enabled() else None
        bl = bias_grad_link()
        x = self.norm1(self.self_attn(x, causal, key_padding_mask, link=link, blink=bl), residual=x, dropout_p=p1,
                       link=link, blink=bl)
        link = residual_link(x) if torch.is_grad_enabled() else None
        bl = bias_grad_link()
        return self.norm2(self._ff(x, link=link, blink=bl), residual=x, dropout_p=p2, link=link, blink=bl)


class TransformerEncoder(nn.Module):
    """Stack of encoder layers (``layers.N.*`` keys), optional activation checkpointing.

    ``use_checkpoint=True`` recomputes each layer in backward (the reference's
    ``checkpoint_sequential(self.transformer.layers, n_layers, x)``,
    ``memory_optimization.ipynb:194-228``; here non-reentrant, per layer).
    """

    def __init__(self, layer_fn, num_layers: int, norm: Optional[nn.Module] = None, use_checkpoint: bool = False):
        super().__init__()
        self.layers = nn.ModuleList([layer_fn() for _ in range(num_layers)])
        self.num_layers = num_layers
        self.norm = norm
        self.use_checkpoint = use_checkpoint

    def forward(self, x: torch.Tensor, causal: bool = False,
                key_padding_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        for layer in self.layers:
            if self.use_checkpoint and self.training and torch.is_grad_enabled():
                x = checkpoint(layer, x, causal, key_padding_mask, use_reentrant=False)
            else:
                x = layer(x, causal, key_padding_mask)
        return self.norm(x) if self.norm is not None else x


def encoder(d_model: int, nhead: int, num_layers: int, dim_feedforward: int = 2048, dropout: float = 0.1,
            activation: str = "relu", norm_first: bool = False, use_checkpoint: bool = False) -> TransformerEncoder:
    return TransformerEncoder(
        lambda: TransformerEncoderLayer(d_model, nhead, dim_feedforward, dropout, activation, norm_first=norm_first),
        num_layers,
        use_checkpoint=use_checkpoint,
    )


class CustomTransformer(nn.Module):
    """The baseline's encoder-only benchmark model (``create_custom_transformer``, C5).

    Input ``[B, S, d_model]`` floats (``batch_first=True``); 6 × post-LN layers, d=512, h=8,
    ff=2048, ReLU, dropout 0.1 — 18.9M parameters.  Keys ``transformer_encoder.layers.N.*``.
    """

    def __init__(self, d_model: int = 512, nhead: int = 8, num_layers: int = 6, dim_feedforward: int = 2048,
                 dropout: float = 0.1, use_checkpoint: bool = False):
        super().__init__()
        self.transformer_encoder = encoder(d_model, nhead, num_layers, dim_feedforward, dropout,
                                           use_checkpoint=use_checkpoint)

    def forward(self, src: torch.Tensor) -> torch.Tensor:
        return self.transformer_encoder(src)


def create_custom_transformer(vocab_size: int = 30000, d_model: int = 512, nhead: int = 8,
                              num_layers: int = 6) -> CustomTransformer:
    """Reference factory signature (``baseline_performance.ipynb:238``); ``vocab_size`` is unused there too."""
    del vocab_size
    return CustomTransformer(d_model=d_model, nhead=nhead, num_layers=num_layers)


def count_params(m: nn.Module) -> int:
    return sum(p.numel() for p in m.parameters())

