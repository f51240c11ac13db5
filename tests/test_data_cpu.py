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
