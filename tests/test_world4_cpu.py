"""Multi-process parity at the reference's world size (4 GCDs, ``data/distributed/*_4gpus_*``) and
at 8 ranks — VERDICT r05 next #3c.  gloo ranks on the CPU run the same DDP bucket / hook code the
segmented GPU schedule issues from (``segments.eager`` executes a hole immediately outside a
capture) and the same FSDP flat-shard, ring-slot and replicate-frozen code.

* DDP at world 4: bucketed all-reduce from the backward hooks, bucket order identical on every rank,
  replicas bit-identical, equal to single-process training on the same 4 quarter-batches;
* FSDP ring at world 4 with 5 units through 2-3 slots (units evict each other every step);
* FSDP at world 8: every flat group padded to a multiple of 8 x 64 elements (aligned shards);
* LoRA-style frozen base with ``replicate_frozen`` at world 4, vs fully sharded;
* sharded checkpoint round trip at world 4.
"""
import pytest
import torch

from dist_utils import run_world
from test_fsdp_cpu import _fsdp_train, _reference_train, _sharded_roundtrip


def _cnn(seed=0):
    from hyperion.models.resnet import resnet18

    torch.manual_seed(seed)
    return resnet18(num_classes=10)


def _data(step, n=16):
    g = torch.Generator().manual_seed(70 + step)
    return torch.randn(n, 3, 32, 32, generator=g), torch.randint(0, 10, (n,), generator=g)


def _ddp_ref(steps, world):
    m = _cnn()
    m.train()
    opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
    per = 16 // world
    for s in range(steps):
        x, y = _data(s)
        # per-rank BN statistics: the mean of the per-rank losses over the rank slices
        loss = sum(torch.nn.functional.cross_entropy(m(x[r * per:(r + 1) * per]), y[r * per:(r + 1) * per])
                   for r in range(world)) / world
        loss.backward()
        opt.step()
        opt.zero_grad()
    return {k: v for k, v in m.state_dict().items() if "running" not in k and "num_batches" not in k}


def _ddp_world(rank, world, steps):
    from hyperion.parallel import DDP

    m = DDP(_cnn(seed=rank), bucket_cap_mb=1.0, first_bucket_mb=0.1, broadcast_buffers=False)
    opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
    order = []
    orig = m.comm.all_reduce

    def spy(t, *a, **k):  # the order in which this rank issues its bucket all-reduces
        order.append(t.numel())
        return orig(t, *a, **k)

    m.comm.all_reduce = spy
    per = 16 // world
    for s in range(steps):
        x, y = _data(s)
        torch.nn.functional.cross_entropy(m(x[rank * per:(rank + 1) * per]), y[rank * per:(rank + 1) * per]).backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
    sd = {k: v for k, v in m.state_dict().items() if "running" not in k and "num_batches" not in k}
    return {"sd": sd, "order": order, "buckets": m.bucket_sizes()}


def test_ddp_world4_matches_single_process_and_bucket_order():
    ref = _ddp_ref(2, 4)
    res = run_world(_ddp_world, 4, (2,), timeout=600)
    assert len(res[0]["buckets"]) > 4
    for r in range(1, 4):
        assert res[r]["order"] == res[0]["order"]  # every rank issues the buckets in the same order
        for k in ref:
            torch.testing.assert_close(res[r]["sd"][k], res[0]["sd"][k], rtol=0, atol=0, msg=k)
    for k in ref:
        torch.testing.assert_close(res[0]["sd"][k], ref[k], rtol=1e-4, atol=1e-5, msg=k)


@pytest.mark.parametrize("ring", [2, 3])
def test_fsdp_ring_world4_more_units_than_slots(ring):
    ref = _reference_train(2, clip=0.05, layers=5)
    res = run_world(_fsdp_train, 4, (2, "layer", 0.05, "FULL_SHARD", None, ring, 5), timeout=600)
    assert res[0]["plan"]["mode"] == f"ring{ring}" and len(res[0]["units"]) == 6  # 5 layers + root
    for k in ref:
        torch.testing.assert_close(res[0]["sd"][k], ref[k], rtol=1e-4, atol=1e-5, msg=k)


def _padding_world(rank, world):
    from hyperion.models.transformer import TransformerEncoderLayer
    from hyperion.parallel.fsdp import FSDP, transformer_auto_wrap_policy
    from test_fsdp_cpu import _batch, _make_model

    m = FSDP(_make_model(), auto_wrap_policy=transformer_auto_wrap_policy({TransformerEncoderLayer}),
             device_id=torch.device("cpu"))
    groups = [(g.numel, g.padded, g.shard_numel, g.flat_param.numel()) for g in m.flat_groups()]
    opt = torch.optim.SGD(m.parameters(), lr=1e-1, momentum=0.9, weight_decay=0.01)
    for s in range(2):
        x, y = _batch(s)
        m.forward_loss(x[rank:rank + 1], y[rank:rank + 1], ignore_index=-100).backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
    return {"groups": groups, "sd": m.full_state_dict(rank0_only=True)}


def test_fsdp_world8_shard_padding_and_parity():
    res = run_world(_padding_world, 8, (), timeout=600)
    for numel, padded, shard, local in res[0]["groups"]:
        assert padded % (8 * 64) == 0 and padded >= numel and padded - numel < 8 * 64
        assert shard == padded // 8 == local
    ref = _reference_train(2)
    for k in ref:
        torch.testing.assert_close(res[0]["sd"][k], ref[k], rtol=1e-4, atol=1e-5, msg=k)


def _lora_world(rank, world, replicate):
    from hyperion.models.transformer import TransformerEncoderLayer
    from hyperion.parallel.fsdp import FSDP, transformer_auto_wrap_policy
    from test_fsdp_cpu import _batch, _make_model

    m0 = _make_model()
    for n, p in m0.named_parameters():
        if "linear1" not in n:  # a frozen base with trainable adapters (the LoRA shape of the problem)
            p.requires_grad_(False)
    m = FSDP(m0, auto_wrap_policy=transformer_auto_wrap_policy({TransformerEncoderLayer}),
             device_id=torch.device("cpu"), replicate_frozen=replicate)
    opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-2)
    per = 8 // world
    for step in range(2):
        x, y = _batch(step)
        opt.zero_grad()
        m.forward_loss(x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per], ignore_index=-100).backward()
        opt.step()
    return {"sd": m.full_state_dict(rank0_only=False), "resident": [g.resident for g in m.flat_groups() if not g.trainable]}


def test_lora_fsdp_replicate_frozen_world4():
    shard = run_world(_lora_world, 4, (False,), timeout=600)
    repl = run_world(_lora_world, 4, (True,), timeout=600)
    assert all(repl[0]["resident"]) and not any(shard[0]["resident"])
    for k in shard[0]["sd"]:
        torch.testing.assert_close(repl[0]["sd"][k], shard[0]["sd"][k], rtol=1e-5, atol=1e-6, msg=k)
        for r in range(1, 4):
            assert torch.equal(repl[r]["sd"][k], repl[0]["sd"][k]), k


def test_fsdp_sharded_checkpoint_roundtrip_world4(tmp_path):
    res = run_world(_sharded_roundtrip, 4, (str(tmp_path),), timeout=600)
    assert all(res[r] for r in range(4))
