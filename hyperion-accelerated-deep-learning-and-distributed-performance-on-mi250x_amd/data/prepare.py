"""Dataset preparation: WikiText-2 tokenization and CIFAR-10 conversion.

Reference: ``02_development/dataset_preparation.ipynb`` —

* WikiText-2 (:161-221): ``load_dataset("wikitext", "wikitext-2-raw-v1")``, drop empty lines
  (36718→23767 train, 4358→2891 test, 3760→2461 validation), GPT-2 fast tokenizer with
  ``pad_token = eos`` (50256), ``truncation=True, padding="max_length", max_length=128``,
  attention mask, ``save_to_disk`` → ``data/processed/wikitext2_tokenized`` (``input_ids`` int32,
  ``attention_mask`` int8, per split).
* CIFAR-10 (:282-338): torchvision CIFAR10 + ``ToTensor()`` + ``Normalize(0.5, 0.5)``, drop invalid
  or all-zero images, ``torch.save(list[(Tensor[3,32,32], int)])`` → ``cifar10_{train,test}.pt``.

This container has no network, so nothing is downloaded: ``prepare_wikitext2`` takes the raw
lines per split (e.g. read from a local copy of the wikitext raw files) and any tokenizer callable
(``transformers`` GPT-2 tokenizer when its files are cached locally; ``HashTokenizer`` otherwise —
a deterministic offline stand-in with the GPT-2 vocabulary size and pad id), and
``prepare_cifar10`` reads the CIFAR-10 *binary* distribution (``data_batch_*.bin``: 1 label byte
+ 3072 pixel bytes per record — plain bytes, no pickle).  Outputs use the reference's layout, so
``load_wikitext2`` / ``load_cifar10_pt`` and the trainers read them unchanged.
"""
from __future__ import annotations

import os
import re
import zlib
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

GPT2_VOCAB = 50257
GPT2_EOS = 50256


class HashTokenizer:
    """Offline stand-in for the GPT-2 tokenizer: words/punctuation → crc32 ids in [0, 50256).

    Same call signature as a HF tokenizer for the reference's usage:
    ``tok(texts, truncation=True, padding="max_length", max_length=128)`` →
    ``{"input_ids": [[...]], "attention_mask": [[...]]}`` with pad = eos = 50256.
    """

    pad_token_id = GPT2_EOS
    eos_token_id = GPT2_EOS
    vocab_size = GPT2_VOCAB
    _pat = re.compile(r"\w+|[^\w\s]")

    def encode(self, text: str) -> List[int]:
        return [zlib.crc32(t.encode()) % GPT2_EOS for t in self._pat.findall(text)]

    def __call__(self, texts, truncation: bool = True, padding: str = "max_length", max_length: int = 128, **_):
        single = isinstance(texts, str)
        ids, masks = [], []
        for t in [texts] if single else texts:
            x = self.encode(t)
            if truncation:
                x = x[:max_length]
            m = [1] * len(x)
            if padding == "max_length" and len(x) < max_length:
                m += [0] * (max_length - len(x))
                x += [self.pad_token_id] * (max_length - len(x))
            ids.append(x)
            masks.append(m)
        return {"input_ids": ids[0] if single else ids, "attention_mask": masks[0] if single else masks}


def gpt2_tokenizer(local_only: bool = True):
    """The reference's tokenizer (``AutoTokenizer.from_pretrained("gpt2")``, pad = eos) when cached
    locally, else :class:`HashTokenizer`."""
    try:
        from transformers import AutoTokenizer

        tok = AutoTokenizer.from_pretrained("gpt2", local_files_only=local_only)
        tok.pad_token = tok.eos_token
        return tok
    except Exception:  # noqa: BLE001 - no cached files / no network
        return HashTokenizer()


def filter_nonempty(lines: Iterable[str]) -> List[str]:
    """The reference's filter: keep lines with non-whitespace content (``len(x["text"].strip()) > 0``)."""
    return [ln for ln in lines if ln.strip()]


def tokenize_lines(lines: Sequence[str], tokenizer: Callable, max_length: int = 128,
                   batch: int = 1000) -> Dict[str, np.ndarray]:
    ids, mask = [], []
    for i in range(0, len(lines), batch):
        enc = tokenizer(list(lines[i:i + batch]), truncation=True, padding="max_length", max_length=max_length)
        ids.extend(enc["input_ids"])
        mask.extend(enc["attention_mask"])
    return {"input_ids": np.asarray(ids, dtype=np.int32).reshape(-1, max_length),
            "attention_mask": np.asarray(mask, dtype=np.int8).reshape(-1, max_length)}


def prepare_wikitext2(raw: Dict[str, Sequence[str]], out_dir: str, tokenizer: Optional[Callable] = None,
                      max_length: int = 128) -> Dict[str, int]:
    """Filter + tokenize each split and ``save_to_disk`` (HF DatasetDict layout) under ``out_dir``.

    ``raw``: ``{"train": lines, "test": lines, "validation": lines}`` (any subset).  Returns the
    kept row count per split (the reference printed 23767 / 2891 / 2461 for the real corpus)."""
    import datasets

    tok = tokenizer or gpt2_tokenizer()
    splits, counts = {}, {}
    for name, lines in raw.items():
        kept = filter_nonempty(lines)
        enc = tokenize_lines(kept, tok, max_length)
        splits[name] = datasets.Dataset.from_dict(
            {"input_ids": enc["input_ids"].tolist(), "attention_mask": enc["attention_mask"].tolist()},
            features=datasets.Features({"input_ids": datasets.Sequence(datasets.Value("int32")),
                                        "attention_mask": datasets.Sequence(datasets.Value("int8"))}))
        counts[name] = len(kept)
    os.makedirs(out_dir, exist_ok=True)
    datasets.DatasetDict(splits).save_to_disk(out_dir)
    return counts


def read_wikitext_raw(path: str) -> List[str]:
    """Lines of a local ``wiki.{train,valid,test}.raw`` file (the raw WikiText-2 distribution)."""
    with open(path, encoding="utf-8") as f:
        return f.read().split("\n")


def read_cifar10_bin(paths: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
    """CIFAR-10 binary records → (uint8 images [N, 3, 32, 32], int64 labels [N])."""
    recs = [np.fromfile(p, dtype=np.uint8).reshape(-1, 3073) for p in paths]
    r = np.concatenate(recs) if recs else np.zeros((0, 3073), np.uint8)
    return r[:, 1:].reshape(-1, 3, 32, 32), r[:, 0].astype(np.int64)


def to_normalized_pairs(images: np.ndarray, labels: np.ndarray) -> List[Tuple[torch.Tensor, int]]:
    """``ToTensor() + Normalize((0.5,)*3, (0.5,)*3)`` and the reference's validity filter (drop
    images with non-finite values or all zeros before normalization)."""
    out = []
    for img, lab in zip(images, labels):
        x = torch.from_numpy(img.astype(np.float32) / 255.0)
        if not torch.isfinite(x).all() or float(x.abs().sum()) == 0.0 or not (0 <= int(lab) < 10):
            continue
        out.append(((x - 0.5) / 0.5, int(lab)))
    return out


def prepare_cifar10(bin_dir: str, out_dir: str) -> Dict[str, int]:
    """``data_batch_{1..5}.bin`` / ``test_batch.bin`` → ``cifar10_{train,test}.pt`` (reference layout)."""
    os.makedirs(out_dir, exist_ok=True)
    counts = {}
    for split, names in (("train", [f"data_batch_{i}.bin" for i in range(1, 6)]), ("test", ["test_batch.bin"])):
        paths = [os.path.join(bin_dir, n) for n in names if os.path.exists(os.path.join(bin_dir, n))]
        if not paths:
            continue
        pairs = to_normalized_pairs(*read_cifar10_bin(paths))
        torch.save(pairs, os.path.join(out_dir, f"cifar10_{split}.pt"))
        counts[split] = len(pairs)
    return counts
