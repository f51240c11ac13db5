"""Synthetic datasets with the shapes of the reference's real data (no network here).

* ``SyntheticWikiText2`` — GPT-2-tokenized WikiText-2 as prepared by
  ``dataset_preparation.ipynb:193-209``: ``input_ids`` int [128] padded with 50256 (pad = eos),
  ``attention_mask`` [128].  Real lines are short: lengths are drawn from a clipped log-normal so
  the pad fraction resembles the real set (most rows are mostly padding), which matters for the
  ``ignore_index=pad`` loss.  Default size 23,767 = the filtered train split (:72-88).
* ``SyntheticCIFAR10`` — 3×32×32 normalised to [-1, 1] (``Normalize(0.5, 0.5)``, :282-311), 10
  classes, 50,000 images.
* ``SyntheticImageNet`` — 3×224×224 ``torch.rand`` images with (B, 1000) ``torch.rand`` targets, the
  baseline benchmark's inputs (``baseline_performance.ipynb:278-279``).

All generators are seeded and produce the whole epoch deterministically per index, so DDP ranks
see disjoint, reproducible shards through ``DistributedSampler``.
"""
from __future__ import annotations

import torch
from torch.utils.data import Dataset

from ..models.simple_lm import GPT2_PAD, GPT2_VOCAB

WIKITEXT2_TRAIN_ROWS = 23767
WIKITEXT2_SEQ = 128
CIFAR10_TRAIN = 50000


class SyntheticWikiText2(Dataset):
    def __init__(self, n: int = WIKITEXT2_TRAIN_ROWS, seq_len: int = WIKITEXT2_SEQ, vocab: int = GPT2_VOCAB,
                 pad_id: int = GPT2_PAD, seed: int = 0, full_length: bool = False):
        g = torch.Generator().manual_seed(seed)
        if full_length:
            lengths = torch.full((n,), seq_len, dtype=torch.long)
        else:
            # WikiText-2 non-empty lines: median ≈ 25 GPT-2 tokens, long tail past 128
            ln = torch.exp(torch.randn(n, generator=g) * 0.9 + 3.2)
            lengths = ln.round().clamp(2, seq_len).long()
        ids = torch.randint(0, vocab - 1, (n, seq_len), generator=g)
        pos = torch.arange(seq_len)[None, :]
        mask = (pos < lengths[:, None]).long()
        self.input_ids = torch.where(mask.bool(), ids, torch.full_like(ids, pad_id))
        self.attention_mask = mask

    def __len__(self) -> int:
        return self.input_ids.shape[0]

    def __getitem__(self, i: int):
        return self.input_ids[i], self.attention_mask[i]

    def tensors(self):
        return self.input_ids, self.attention_mask


class SyntheticCIFAR10(Dataset):
    def __init__(self, n: int = CIFAR10_TRAIN, num_classes: int = 10, image: int = 32, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        self.x = torch.rand(n, 3, image, image, generator=g) * 2 - 1
        self.y = torch.randint(0, num_classes, (n,), generator=g)

    def __len__(self) -> int:
        return self.x.shape[0]

    def __getitem__(self, i: int):
        return self.x[i], int(self.y[i])

    def tensors(self):
        return self.x, self.y


class SyntheticImageNet(Dataset):
    """``torch.rand`` images + regression targets (the reference benchmark's MSE setup) or labels."""

    def __init__(self, n: int = 1024, image: int = 224, num_classes: int = 1000, regression: bool = True,
                 seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        self.x = torch.rand(n, 3, image, image, generator=g)
        self.y = torch.rand(n, num_classes, generator=g) if regression else torch.randint(0, num_classes, (n,),
                                                                                          generator=g)

    def __len__(self) -> int:
        return self.x.shape[0]

    def __getitem__(self, i: int):
        return self.x[i], self.y[i]

    def tensors(self):
        return self.x, self.y
