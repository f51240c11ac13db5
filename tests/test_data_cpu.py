"""Data pipeline: sampler parity with torch, dataset wrappers, the reference's real arrow data."""
import os

import pytest
import torch
import torch.utils.data as tud

from hyperion.data import (DistributedSampler, SyntheticCIFAR10, SyntheticWikiText2, WikiText2TorchDataset,
                           load_wikitext2)

REF_WT2 = "/root/reference/data/wikitext2_tokenized"


@pytest.mark.parametrize("n,world,shuffle,drop_last", [(10, 3, True, False), (10, 3, False, False), (11, 4, True, True),
                                                       (2, 4, True, False), (100, 8, True, False)])
def test_sampler_matches_torch(n, world, shuffle, drop_last):
    ds = list(range(n))
    for epoch in (0, 3):
        for rank in range(world):
            a = DistributedSampler(ds, world, rank, shuffle=shuffle, seed=7, drop_last=drop_last)
            b = tud.DistributedSampler(ds, world, rank, shuffle=shuffle, seed=7, drop_last=drop_last)
            a.set_epoch(epoch)
            b.set_epoch(epoch)
            assert list(a) == list(b)
            assert len(a) == len(b)


def test_sampler_shards_cover_dataset():
    ds = list(range(37))
    seen = []
    for r in range(4):
        seen += list(DistributedSampler(ds, 4, r))
    assert set(seen) == set(range(37)) and len(seen) == 40


def test_synthetic_wikitext_shapes_and_pad_mix():
    ds = SyntheticWikiText2(n=500, seed=1)
    ids, m = ds[0]
    assert ids.shape == (128,) and m.shape == (128,) and ids.dtype == torch.long
    pad_frac = (ds.input_ids == 50256).float().mean().item()
    assert 0.5 < pad_frac < 0.95
    assert torch.equal((ds.input_ids != 50256).long(), ds.attention_mask)
    again = SyntheticWikiText2(n=500, seed=1)
    assert torch.equal(ds.input_ids, again.input_ids)


def test_synthetic_cifar():
    ds = SyntheticCIFAR10(n=16)
    x, y = ds[3]
    assert x.shape == (3, 32, 32) and 0 <= y < 10 and x.min() >= -1 and x.max() <= 1


def test_wikitext_wrapper_over_dict_and_dataset():
    d = {"input_ids": [[1, 2, 3]], "attention_mask": [[1, 1, 0]]}
    ds = WikiText2TorchDataset(d)
    ids, m = ds[0]
    assert ids.tolist() == [1, 2, 3] and m.tolist() == [1, 1, 0]


@pytest.mark.skipif(not os.path.isdir(REF_WT2), reason="reference data not present")
def test_reference_arrow_test_split_loads():
    # the reference snapshot holds the tokenized test/validation splits (train arrow is missing)
    ds = load_wikitext2(REF_WT2, "test")
    w = WikiText2TorchDataset(ds, split="test")
    assert len(w) == 2891  # dataset_preparation.ipynb:72-88 (non-empty test lines)
    ids, m = w[0]
    assert ids.shape == (128,) and m.shape == (128,)
    assert int(ids[m == 0][0]) == 50256 if (m == 0).any() else True


def test_prepare_wikitext2_roundtrip(tmp_path):
    """C11: filter empty lines, tokenize to 128 with pad = eos, save_to_disk, read back with the
    reference wrapper."""
    from hyperion.data.datasets import WikiText2TorchDataset, load_wikitext2
    from hyperion.data.prepare import HashTokenizer, prepare_wikitext2

    raw = {"train": ["", " = Title = ", "   ", "some words, more words .", ""] * 3, "test": ["", "x y"]}
    counts = prepare_wikitext2(raw, str(tmp_path / "wt2"), tokenizer=HashTokenizer())
    assert counts == {"train": 6, "test": 1}
    ds = WikiText2TorchDataset(load_wikitext2(str(tmp_path / "wt2"), "train"))
    assert len(ds) == 6
    ids, mask = ds[0]
    assert ids.shape == (128,) and ids.dtype == torch.long and mask.dtype == torch.long
    assert int(mask.sum()) == 3 and int(ids[-1]) == 50256  # "= Title =" -> 3 tokens, then eos padding


def test_prepare_cifar10_binary(tmp_path):
    """C12: CIFAR-10 binary records -> normalized (Tensor[3,32,32], label) list, all-zero image dropped."""
    import numpy as np

    from hyperion.data.datasets import load_cifar10_pt
    from hyperion.data.prepare import prepare_cifar10

    rng = np.random.default_rng(0)
    recs = rng.integers(0, 256, size=(5, 3073), dtype=np.uint8)
    recs[:, 0] = [0, 3, 9, 1, 2]
    recs[2, 1:] = 0  # all-zero image: filtered like the reference
    recs.tofile(tmp_path / "data_batch_1.bin")
    recs[:2].tofile(tmp_path / "test_batch.bin")
    counts = prepare_cifar10(str(tmp_path), str(tmp_path / "out"))
    assert counts == {"train": 4, "test": 2}
    pairs = load_cifar10_pt(str(tmp_path / "out" / "cifar10_train.pt"))
    x, y = pairs[0]
    assert x.shape == (3, 32, 32) and y == 0 and float(x.min()) >= -1.0 and float(x.max()) <= 1.0


def test_device_tensor_loader_matches_dataloader_batches():
    """DeviceTensorLoader (whole dataset resident, batched by index_select) yields exactly the
    DataLoader's batches for the same DistributedSampler — every rank, every epoch, short last batch."""
    import torch
    from torch.utils.data import DataLoader

    from hyperion.data import DistributedSampler, SyntheticCIFAR10, SyntheticWikiText2
    from hyperion.data.loader import DeviceTensorLoader, dataset_tensors

    for ds in (SyntheticWikiText2(n=70, seed=3), SyntheticCIFAR10(n=70, seed=3)):
        for rank in (0, 1):
            s = DistributedSampler(ds, num_replicas=2, rank=rank, shuffle=True, seed=5)
            dev = DeviceTensorLoader(dataset_tensors(ds), s, 8, torch.device("cpu"))
            ref = DataLoader(ds, batch_size=8, sampler=s)
            for ep in (0, 1):
                s.set_epoch(ep)
                a, b = list(dev), list(ref)
                assert len(a) == len(b) == len(dev)
                for x, y in zip(a, b):
                    assert all(torch.equal(u, torch.as_tensor(v)) for u, v in zip(x, y))
