"""Token embedding on gfx950 (``csrc/kernels/embedding.hip``).

Reference: ``nn.Embedding`` in SimpleTransformerLM (V = 50257) and HF Llama ``embed_tokens``
(V = 32000) — index_select forward, ``embedding_dense_backward`` (SURVEY §2.4 "Embedding").
``Embedding`` keeps ``nn.Embedding``'s parameters, keys and ``padding_idx`` semantics (the pad row
gets no gradient); on GPU the forward is a vectorized row gather and the backward accumulates
token rows with full-rate fp32 atomics (one 256-byte run per wave instruction) into a zeroed
buffer, cast once to the weight dtype.  ``max_norm`` / ``scale_grad_by_freq`` / ``sparse`` fall back to PyTorch.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native


class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w, pad_idx):
        ids = ids.contiguous()
        ctx.save_for_backward(ids)
        ctx.meta = (w.shape[0], pad_idx)
        return _native.native().embedding_fwd(ids, w)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        V, pad = ctx.meta
        dw = _native.native().embedding_bwd(dy.contiguous(), ids, V, pad)
        return None, dw, None


def embedding(ids: torch.Tensor, w: torch.Tensor, padding_idx: Optional[int] = None) -> torch.Tensor:
    if (w.is_cuda and w.dim() == 2 and w.shape[1] % 8 == 0 and w.is_contiguous() and ids.dtype == torch.long
            and w.dtype in (torch.bfloat16, torch.float16, torch.float32) and _native.use_native(w, op="embedding")):
        pad = -1 if padding_idx is None else (padding_idx if padding_idx >= 0 else padding_idx + w.shape[0])
        return _native.apply_fn(_EmbedFn, ids, w, pad)
    return F.embedding(ids, w, padding_idx)


class Embedding(nn.Embedding):
    def forward(self, ids: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        if self.max_norm is not None or self.scale_grad_by_freq or self.sparse:
            return super().forward(ids)
        return embedding(ids, self.weight, self.padding_idx)
