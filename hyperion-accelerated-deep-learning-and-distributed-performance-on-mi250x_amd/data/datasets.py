"""Dataset wrappers with the reference's API (C13) plus real-data adapters (C11, C12).

Reference: ``WikiText2TorchDataset(hf_dataset, split)`` returns ``(input_ids long[128],
attention_mask long[128])`` and ``CIFAR10TorchDataset(data)`` wraps a list of ``(img, label)``
(``02_development/distributed_utils.py:43-67``; duplicated in three notebooks).  The preprocessed
artefacts they read are an HF ``save_to_disk`` directory (``data/processed/wikitext2_tokenized``,
``dataset_preparation.ipynb:207-209``) and ``torch.save``d lists ``cifar10_{train,test}.pt``
(:331-332).

Loading rules here: arrow data through ``datasets.load_from_disk`` (or pyarrow directly), ``.pt``
lists only through ``torch.load(weights_only=True)`` — nothing that unpickles arbitrary objects.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch
from torch.utils.data import Dataset


class WikiText2TorchDataset(Dataset):
    """``hf_dataset`` is a ``DatasetDict`` (indexed by ``split``) or a single split / column mapping."""

    def __init__(self, hf_dataset, split: str = "train"):
        ds = hf_dataset
        try:
            if split is not None and hasattr(ds, "keys") and split in ds.keys():
                ds = ds[split]
        except TypeError:
            pass
        self.ds = ds
        self._ids = None
        self._mask = None
        cols = getattr(ds, "column_names", None)
        if cols is None and isinstance(ds, dict):
            self._ids = ds["input_ids"]
            self._mask = ds.get("attention_mask")

    def __len__(self) -> int:
        return len(self._ids) if self._ids is not None else len(self.ds)

    def __getitem__(self, i: int) -> Tuple[torch.Tensor, torch.Tensor]:
        if self._ids is not None:
            ids, m = self._ids[i], (self._mask[i] if self._mask is not None else None)
        else:
            rec = self.ds[i]
            ids, m = rec["input_ids"], rec.get("attention_mask")
        ids = torch.as_tensor(ids, dtype=torch.long)
        m = torch.ones_like(ids) if m is None else torch.as_tensor(m, dtype=torch.long)
        return ids, m

    def tensors(self):
        """[N, 128] token ids and mask (fixed-length rows: the tokenizer padded to max_length)."""
        if self._ids is not None:
            ids = torch.as_tensor(self._ids, dtype=torch.long)
            m = torch.ones_like(ids) if self._mask is None else torch.as_tensor(self._mask, dtype=torch.long)
            return ids, m
        cols = self.ds.with_format("torch")  # HF datasets: columnar, no per-sample Python
        ids = cols["input_ids"].long()
        m = cols["attention_mask"].long() if "attention_mask" in self.ds.column_names else torch.ones_like(ids)
        return ids, m


class CIFAR10TorchDataset(Dataset):
    def __init__(self, data: Sequence):
        self.data = data

    def __len__(self) -> int:
        return len(self.data)

    def __getitem__(self, i: int):
        img, label = self.data[i]
        return img, label

    def tensors(self):
        return torch.stack([d[0] for d in self.data]), torch.as_tensor([int(d[1]) for d in self.data])


class TensorPairDataset(Dataset):
    """Pre-materialised ``(x, y)`` tensors (synthetic sets live here)."""

    def __init__(self, x: torch.Tensor, y: torch.Tensor):
        assert len(x) == len(y)
        self.x, self.y = x, y

    def __len__(self) -> int:
        return len(self.x)

    def __getitem__(self, i: int):
        return self.x[i], self.y[i]

    def tensors(self):
        return self.x, self.y


def load_wikitext2(path: str, split: Optional[str] = None):
    """Load the reference's tokenized WikiText-2 (HF ``save_to_disk`` layout).

    ``path`` may be the ``DatasetDict`` root or one split directory.  Returns a ``datasets``
    object; falls back to reading the arrow file with pyarrow when ``load_from_disk`` refuses
    a partial dict (the reference snapshot is missing its train split).
    """
    if split is not None and os.path.isdir(os.path.join(path, split)):
        path = os.path.join(path, split)
    try:
        import datasets

        return datasets.load_from_disk(path)
    except Exception:
        return _read_arrow_columns(path)


def _read_arrow_columns(path: str) -> dict:
    import glob

    import pyarrow as pa

    files = sorted(glob.glob(os.path.join(path, "*.arrow")))
    if not files:
        raise FileNotFoundError(f"no .arrow files under {path}")
    tables = []
    for f in files:
        with pa.memory_map(f, "r") as src:
            try:
                tables.append(pa.ipc.open_stream(src).read_all())
            except pa.ArrowInvalid:
                tables.append(pa.ipc.open_file(src).read_all())
    t = pa.concat_tables(tables)
    return {c: t.column(c).to_pylist() for c in t.column_names}


def load_cifar10_pt(path: str) -> List[Tuple[torch.Tensor, int]]:
    """Load a ``cifar10_{train,test}.pt`` list with the safe loader (``weights_only=True``)."""
    data = torch.load(path, map_location="cpu", weights_only=True)
    return [(img, int(lbl)) for img, lbl in data]
