"""SimpleTransformerLM — the reference's language model, in both of its key layouts.

Reference definitions:
* distributed trainers (C14): ``Embedding(V, 256) → TransformerEncoder(TransformerEncoderLayer(256,
  nhead=4), 2) → Linear(256, V)`` with attributes ``embed / tr / fc`` —
  ``02_development/distributed_utils.py:75-88``;
* notebooks (C14/C16): the same network with attributes ``embedding / transformer / fc`` and a
  ``max_len`` / ``use_checkpoint`` argument — ``core_framework.ipynb:185-200``,
  ``memory_optimization.ipynb:194-228``;
* compile bench (C15): 768-d, 12 heads, ff 3072, GELU, 4 layers, input ``idx`` as ``[T, B]`` —
  ``compilation_optimization.py:57-71``.

Reference behaviour kept for metric parity: no causal mask and no padding mask;
``causal=True`` turns on a proper LM mask.  The reference's ``permute`` to sequence-first and
back is dropped (the encoder runs batch-major, see ``models/transformer.py``).

``forward(ids)`` returns logits like the reference.  ``forward_loss(ids, targets)`` is the fast
training path: the ``fc`` head and the cross-entropy are one fused op
(``ops.cross_entropy.fused_linear_cross_entropy``), so the [B·S, V] fp32 log-prob tensor of the
reference never exists.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from ..ops.embedding import Embedding
from ..ops.cross_entropy import LinearCrossEntropy
from .transformer import encoder

GPT2_VOCAB = 50257
GPT2_PAD = 50256  # GPT-2 tokenizer with pad = eos (dataset_preparation.ipynb:193-204)


class SimpleTransformerLM(nn.Module):
    """``key_style='ddp'`` → ``embed/tr/fc`` (distributed_utils.py); ``'notebook'`` → ``embedding/transformer/fc``."""

    def __init__(
        self,
        vocab_size: int = GPT2_VOCAB,
        emb_dim: int = 256,
        n_heads: int = 4,
        n_layers: int = 2,
        ff_dim: int = 2048,
        activation: str = "relu",
        dropout: float = 0.1,
        max_len: int = 128,
        use_checkpoint: bool = False,
        causal: bool = False,
        key_style: str = "ddp",
        seq_first_input: bool = False,
    ):
        super().__init__()
        if key_style not in ("ddp", "notebook"):
            raise ValueError(f"key_style {key_style!r}")
        self.key_style = key_style
        self._emb_name, self._enc_name = ("embed", "tr") if key_style == "ddp" else ("embedding", "transformer")
        setattr(self, self._emb_name, Embedding(vocab_size, emb_dim))
        setattr(self, self._enc_name, encoder(emb_dim, n_heads, n_layers, ff_dim, dropout, activation,
                                              use_checkpoint=use_checkpoint))
        self.fc = LinearCrossEntropy(emb_dim, vocab_size)
        self.vocab_size = vocab_size
        self.max_len = max_len
        self.causal = causal
        self.seq_first_input = seq_first_input  # the 768-d compile-bench model takes idx [T, B]

    @property
    def use_checkpoint(self) -> bool:
        return getattr(self, self._enc_name).use_checkpoint

    @use_checkpoint.setter
    def use_checkpoint(self, v: bool) -> None:
        getattr(self, self._enc_name).use_checkpoint = bool(v)

    def hidden(self, ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Encoder output ``[B, S, E]`` (batch-major ``ids``); reference ignores ``attention_mask``."""
        del attention_mask  # the reference accepts and ignores it (core_framework.ipynb:194)
        x = getattr(self, self._emb_name)(ids)
        return getattr(self, self._enc_name)(x, causal=self.causal)

    def forward(self, ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                targets: Optional[torch.Tensor] = None, ignore_index: int = GPT2_PAD, **_) -> torch.Tensor:
        """Logits like the reference; with ``targets`` the fused-head mean CE loss (so wrappers that
        only intercept ``forward`` — DDP, FSDP — see the training path too)."""
        if targets is not None:
            return self.forward_loss(ids, targets, ignore_index, attention_mask)
        if self.seq_first_input:
            return self.fc(self.hidden(ids.t(), attention_mask)).transpose(0, 1)
        return self.fc(self.hidden(ids, attention_mask))

    def forward_loss(self, ids: torch.Tensor, targets: torch.Tensor, ignore_index: int = GPT2_PAD,
                     attention_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Mean next-token CE (ignore pads) with the LM head fused into the loss."""
        h = self.hidden(ids, attention_mask)
        return self.fc(h, target=targets, ignore_index=ignore_index)


def simple_lm_256(vocab_size: int = GPT2_VOCAB, **kw) -> SimpleTransformerLM:
    """C14: 28,411,985 parameters at V = 50257."""
    cfg = dict(emb_dim=256, n_heads=4, n_layers=2, ff_dim=2048, activation="relu")
    cfg.update(kw)
    return SimpleTransformerLM(vocab_size, **cfg)


def simple_lm_768(vocab_size: int = GPT2_VOCAB, **kw) -> SimpleTransformerLM:
    """C15 (compile bench): 768-d, 12 heads, ff 3072, GELU, 4 layers, ``[T, B]`` input, notebook keys."""
    kw.setdefault("key_style", "notebook")
    kw.setdefault("seq_first_input", True)
    return SimpleTransformerLM(vocab_size, emb_dim=768, n_heads=12, n_layers=4, ff_dim=3072, activation="gelu", **kw)


def gpt2_small_lm(vocab_size: int = GPT2_VOCAB, **kw) -> SimpleTransformerLM:
    """GPT-2-small-shaped encoder LM (12 × 768, 12 heads, ff 3072, GELU, causal) for the FSDP config."""
    cfg = dict(emb_dim=768, n_heads=12, n_layers=12, ff_dim=3072, activation="gelu", causal=True, dropout=0.1)
    cfg.update(kw)
    return SimpleTransformerLM(vocab_size, **cfg)
