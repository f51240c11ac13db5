"""Multi-tensor pointer tables (ops/multi_tensor.py): a table used by a hipGraph capture is pinned
and never re-pointed by a later eager call (an eager step or a second capture with the
same layout used to redirect the captured Adam / clip kernels to other tensors)."""
import torch

from hyperion.ops import multi_tensor as mt


def _groups(n=3, size=64):
    return [[torch.empty(size, dtype=torch.float32) for _ in range(n)]]


def test_unpinned_table_is_repointed_in_place():
    c = mt.TableCache()
    a, b = _groups(), _groups()
    t1 = c.get("adam", a)
    t2 = c.get("adam", b)
    assert t2 is t1 and t1.key == mt.MultiTensorTable.key_of(b)
    assert t1.ptrs.tolist() == [x.data_ptr() for x in b[0]]


def test_captured_table_is_pinned(monkeypatch):
    c = mt.TableCache()
    warm, captured, eager = _groups(), _groups(), _groups()
    t0 = c.get("adam", warm)
    monkeypatch.setattr(mt, "_capturing", lambda dev: True)
    tc = c.get("adam", captured)  # capture: re-points the warm-up table, and pins it
    monkeypatch.setattr(mt, "_capturing", lambda dev: False)
    assert tc is t0 and getattr(tc, "pinned", False)
    cap_ptrs = tc.ptrs.tolist()
    te = c.get("adam", eager)  # later eager call with other tensors: a table of its own
    assert te is not tc and tc.ptrs.tolist() == cap_ptrs
    assert te.ptrs.tolist() == [x.data_ptr() for x in eager[0]]
    assert c.get("adam", captured) is tc  # the captured set maps back to its pinned table
    assert c.pinned() == [tc]


def test_clip_cache_is_per_model():
    from hyperion.ops import optim

    m1, m2 = torch.nn.Linear(4, 4), torch.nn.Linear(4, 4)
    for m in (m1, m2):
        m.weight.grad = torch.ones_like(m.weight)
        m.bias.grad = torch.ones_like(m.bias)
    optim.clip_grad_norm_(m1.parameters(), 1.0)
    optim.clip_grad_norm_(m2.parameters(), 1.0)
    # CPU tensors take the reference path (no table); the cache is keyed per model, never global
    assert not isinstance(optim._clip_tables, mt.TableCache)
