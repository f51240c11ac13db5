"""FSDP (flat-param FULL_SHARD) on gloo: parity with single-process training, state dicts, LoRA-frozen."""
import copy

import pytest
import torch

from dist_utils import run_world


def _make_model(seed=0, layers=2):
    from hyperion.models.simple_lm import simple_lm_256

    torch.manual_seed(seed)
    return simple_lm_256(vocab_size=64, emb_dim=32, n_heads=2, n_layers=layers, ff_dim=48, dropout=0.0)


def _batch(step, n=8):
    g = torch.Generator().manual_seed(100 + step)
    ids = torch.randint(0, 64, (n, 9), generator=g)
    return ids[:, :-1], ids[:, 1:]


def _reference_train(steps, lr=1e-2, clip=None, layers=2):
    m = _make_model(layers=layers)
    # SGD keeps the comparison strict: Adam would turn the (exactly zero in exact arithmetic) key-bias
    # gradient's rounding noise into +-lr steps that depend on the summation order across ranks
    opt = torch.optim.SGD(m.parameters(), lr=lr * 10, momentum=0.9, weight_decay=0.01)
    for s in range(steps):
        x, y = _batch(s)
        loss = m.forward_loss(x, y, ignore_index=-100)
        loss.backward()
        if clip is not None:
            torch.nn.utils.clip_grad_norm_(m.parameters(), clip)
        opt.step()
        opt.zero_grad()
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


def _fsdp_train(rank, world, steps, policy_kind, clip, strategy, persistent=None, ring=0, layers=2):
    from hyperion.models.transformer import TransformerEncoderLayer
    from hyperion.parallel.fsdp import FSDP, size_based_auto_wrap_policy, transformer_auto_wrap_policy

    policy = {"layer": transformer_auto_wrap_policy({TransformerEncoderLayer}),
              "size": size_based_auto_wrap_policy(2000),
              # every Linear its own unit (the reference's min_num_params=100_000 at full size):
              # the FFN / attention projections must be CALLED as modules for the gather hooks
              "leaf": size_based_auto_wrap_policy(500), "none": None}[policy_kind]
    m = FSDP(_make_model(layers=layers), auto_wrap_policy=policy, device_id=torch.device("cpu"),
             sharding_strategy=strategy, persistent=persistent, ring=ring)
    if ring:  # every ring slot starts poisoned: a unit must never compute from a slot it does not own
        for r in m._rings.values():
            for b in r.bufs:
                b.fill_(float("nan"))
    if persistent:
        for g in m.flat_groups():  # an allocated-but-unfilled full buffer must never be read as gathered
            if not g.resident:
                g.full.fill_(float("nan"))
    opt = torch.optim.SGD(m.parameters(), lr=1e-1, momentum=0.9, weight_decay=0.01)
    per = 8 // world
    for s in range(steps):
        x, y = _batch(s)
        x, y = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
        loss = m.forward_loss(x, y, ignore_index=-100)
        loss.backward()
        if clip is not None:
            m.clip_grad_norm_(clip)
        opt.step()
        opt.zero_grad(set_to_none=True)
    sd = m.full_state_dict(rank0_only=True)
    return {"sd": sd, "units": m.unit_sizes(), "plan": m.memory_plan()}


@pytest.mark.parametrize("policy", ["layer", "size", "leaf", "none"])
@pytest.mark.parametrize("strategy", ["FULL_SHARD", "SHARD_GRAD_OP"])
def test_fsdp_matches_single_process(policy, strategy):
    ref = _reference_train(3)
    res = run_world(_fsdp_train, 2, (3, policy, None, strategy))
    sd = res[0]["sd"]
    assert res[1]["sd"] == {}
    assert set(sd) == set(ref)
    for k in ref:
        torch.testing.assert_close(sd[k], ref[k], rtol=1e-4, atol=1e-5, msg=k)
    if policy == "layer":
        assert len(res[0]["units"]) == 3  # 2 encoder layers + root (embed, fc)


@pytest.mark.parametrize("world", [1, 2])
def test_fsdp_persistent_matches_single_process(world):
    """persistent mode (full params / grad buffers kept allocated, one gather per unit per step): the
    first forward gathers into the fresh buffer (poisoned with NaN here) like every later one."""
    ref = _reference_train(3)
    res = run_world(_fsdp_train, world, (3, "layer", None, "FULL_SHARD", True))
    for k in ref:
        torch.testing.assert_close(res[0]["sd"][k], ref[k], rtol=1e-4, atol=1e-5, msg=k)


@pytest.mark.parametrize("world", [1, 2])
@pytest.mark.parametrize("ring", [2, 3])
def test_fsdp_ring_matches_single_process(world, ring):
    """FULL_SHARD ring mode: 5 layer units share `ring` fixed-address gathered-parameter / gradient
    slots (slots poisoned with NaN first; units evict each other every step, forward and backward,
    with prefetch); training with global clipping matches the single-process reference, and the
    kept buffers are `ring` units' worth, not all five."""
    ref = _reference_train(3, clip=0.05, layers=5)
    res = run_world(_fsdp_train, world, (3, "layer", 0.05, "FULL_SHARD", None, ring, 5))
    for k in ref:
        torch.testing.assert_close(res[0]["sd"][k], ref[k], rtol=1e-4, atol=1e-5, msg=k)
    assert res[0]["plan"]["mode"] == f"ring{ring}"
    per_unit = max(res[0]["units"][:-1])
    assert res[0]["plan"]["gathered_gib"] * 2**30 < (ring + 2) * per_unit * 8  # ring slots + root, fp32 p + g


def test_fsdp_global_grad_clip_matches_single_process():
    ref = _reference_train(3, clip=0.05)
    res = run_world(_fsdp_train, 2, (3, "layer", 0.05, "FULL_SHARD"))
    for k in ref:
        torch.testing.assert_close(res[0]["sd"][k], ref[k], rtol=1e-4, atol=1e-5, msg=k)


def _sharded_roundtrip(rank, world, tmp):
    from hyperion.parallel.fsdp import FSDP, size_based_auto_wrap_policy

    m = FSDP(_make_model(), auto_wrap_policy=size_based_auto_wrap_policy(2000), device_id=torch.device("cpu"))
    sd = m.sharded_state_dict()
    torch.save(sd, f"{tmp}/shard{rank}.pt")
    m2 = FSDP(_make_model(seed=5), auto_wrap_policy=size_based_auto_wrap_policy(2000), device_id=torch.device("cpu"))
    m2.load_sharded_state_dict(torch.load(f"{tmp}/shard{rank}.pt", weights_only=True))
    a = m.full_state_dict(rank0_only=False)
    b = m2.full_state_dict(rank0_only=False)
    # full -> load_full round trip as well
    m3 = FSDP(_make_model(seed=9), device_id=torch.device("cpu"))
    m3.load_full_state_dict(a)
    c = m3.full_state_dict(rank0_only=False)
    return all(torch.equal(a[k], b[k]) and torch.equal(a[k], c[k]) for k in a)


def test_fsdp_sharded_and_full_state_dict_roundtrip(tmp_path):
    res = run_world(_sharded_roundtrip, 2, (str(tmp_path),))
    assert res[0] and res[1]


def _frozen_train(rank, world):
    from hyperion.models.transformer import TransformerEncoderLayer
    from hyperion.parallel.fsdp import FSDP, transformer_auto_wrap_policy

    m0 = _make_model()
    for n, p in m0.named_parameters():
        if "linear1" not in n:
            p.requires_grad_(False)
    before = {k: v.clone() for k, v in m0.state_dict().items()}
    m = FSDP(m0, auto_wrap_policy=transformer_auto_wrap_policy({TransformerEncoderLayer}), device_id=torch.device("cpu"))
    n_opt = sum(p.numel() for p in m.parameters())
    opt = torch.optim.AdamW(m.parameters(), lr=1e-2)
    x, y = _batch(0)
    m.forward_loss(x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4], ignore_index=-100).backward()
    opt.step()
    sd = m.full_state_dict(rank0_only=False)
    changed = {k for k in sd if not torch.equal(sd[k], before[k])}
    return n_opt, changed


def test_fsdp_frozen_params_not_sharded_into_optimizer():
    res = run_world(_frozen_train, 2)
    n_opt, changed = res[0]
    # only linear1 (2 layers x (32*48 + 48)) is trainable; each unit padded to a multiple of
    # world * 64 elements (aligned shards), then sharded over the 2 ranks
    assert (32 * 48 + 48) <= n_opt < (32 * 48 + 48) + 2 * 64
    assert changed and all("linear1" in k for k in changed)


def _replicated_frozen_train(rank, world, replicate):
    from hyperion.models.transformer import TransformerEncoderLayer
    from hyperion.parallel.fsdp import FSDP, transformer_auto_wrap_policy

    m0 = _make_model()
    for n, p in m0.named_parameters():
        if "linear1" not in n:
            p.requires_grad_(False)
    m = FSDP(m0, auto_wrap_policy=transformer_auto_wrap_policy({TransformerEncoderLayer}), device_id=torch.device("cpu"),
             replicate_frozen=replicate)
    gathers = []
    comm_ag = m.comm.all_gather

    def counting_all_gather(out, inp, *a, **k):
        gathers.append(out.numel())
        return comm_ag(out, inp, *a, **k)

    m.comm.all_gather = counting_all_gather
    opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-2)
    for step in range(3):
        x, y = _batch(step)
        opt.zero_grad()
        m.forward_loss(x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4], ignore_index=-100).backward()
        opt.step()
    resident = [g.resident for g in m.flat_groups() if not g.trainable]
    return m.full_state_dict(rank0_only=False), resident, sum(gathers)


def test_fsdp_replicate_frozen_matches_sharded_and_skips_frozen_gathers():
    """replicate_frozen: the frozen base stays whole on every rank (no all-gathers for it), the
    adapters are sharded as usual, and training matches the fully sharded run."""
    shard = run_world(_replicated_frozen_train, 2, (False,))
    repl = run_world(_replicated_frozen_train, 2, (True,))
    sd_s, res_s, ag_s = shard[0]
    sd_r, res_r, ag_r = repl[0]
    assert res_r and all(res_r) and not any(res_s)
    assert ag_r < ag_s  # only the trainable groups are gathered
    for k in sd_s:
        torch.testing.assert_close(sd_r[k], sd_s[k], rtol=1e-5, atol=1e-6)
    for k in sd_r:  # replicas agree
        assert torch.equal(repl[1][0][k], sd_r[k])


def _replicated_roundtrip(rank, world, tmp):
    import os

    from hyperion.models.transformer import TransformerEncoderLayer
    from hyperion.parallel.fsdp import FSDP, transformer_auto_wrap_policy

    def make():
        m0 = _make_model()
        for n, p in m0.named_parameters():
            if "linear1" not in n:
                p.requires_grad_(False)
        return FSDP(m0, auto_wrap_policy=transformer_auto_wrap_policy({TransformerEncoderLayer}),
                    device_id=torch.device("cpu"), replicate_frozen=True)

    m = make()
    want = m.full_state_dict(rank0_only=False)
    sd = m.sharded_state_dict()
    frozen_copies = sum(t is not None for t, g in zip(sd["flat_params"], m.flat_groups()) if g.resident)
    torch.save(sd, os.path.join(tmp, f"s{rank}.pt"))
    torch.distributed.barrier()
    m2 = make()
    with torch.no_grad():
        for g in m2.flat_groups():
            g.flat_param.data.zero_()
    m2.load_sharded_state_dict(torch.load(os.path.join(tmp, f"s{rank}.pt"), weights_only=True))
    got = m2.full_state_dict(rank0_only=False)
    return frozen_copies, all(torch.equal(got[k], want[k]) for k in want)


def test_fsdp_replicated_frozen_sharded_checkpoint_single_copy(tmp_path):
    res = run_world(_replicated_roundtrip, 2, (str(tmp_path),))
    assert res[0][0] > 0 and res[1][0] == 0  # only rank 0 stores the replicated frozen base
    assert res[0][1] and res[1][1]  # and every rank gets it back


def _replicated_roundtrip_subgroup(rank, world, tmp):
    """FSDP over the subgroup {1, 2} (global rank 0 not in it): the replicated frozen base is stored
    by group-rank 0 (global rank 1) and broadcast back from it on load (the broadcast
    used global src=0)."""
    import os

    import torch.distributed as dist

    from hyperion.models.transformer import TransformerEncoderLayer
    from hyperion.parallel.fsdp import FSDP, transformer_auto_wrap_policy

    sub = dist.new_group([1, 2])
    if rank == 0:
        return None

    def make():
        m0 = _make_model()
        for n, p in m0.named_parameters():
            if "linear1" not in n:
                p.requires_grad_(False)
        return FSDP(m0, auto_wrap_policy=transformer_auto_wrap_policy({TransformerEncoderLayer}),
                    device_id=torch.device("cpu"), replicate_frozen=True, process_group=sub)

    m = make()
    want = m.full_state_dict(rank0_only=False)
    sd = m.sharded_state_dict()
    torch.save(sd, os.path.join(tmp, f"s{rank}.pt"))
    dist.barrier(group=sub)
    m2 = make()
    with torch.no_grad():
        for g in m2.flat_groups():
            g.flat_param.data.zero_()
    m2.load_sharded_state_dict(torch.load(os.path.join(tmp, f"s{rank}.pt"), weights_only=True))
    got = m2.full_state_dict(rank0_only=False)
    return all(torch.equal(got[k], want[k]) for k in want)


def test_fsdp_replicated_frozen_subgroup_broadcast_source(tmp_path):
    res = run_world(_replicated_roundtrip_subgroup, 3, (str(tmp_path),))
    assert res[0] is None and res[1] and res[2]


# ---- ring mode: gradient accumulation at world 1 and nested units (medium) ----
def _fsdp_accum_train(rank, world, ring, policy_kind="layer", layers=3, steps=2):
    """Two micro-batch backwards per step and zero_grad(set_to_none=False): .grad exists when the
    second backward's gradients land, so every accumulation path runs."""
    from hyperion.models.transformer import TransformerEncoderLayer
    from hyperion.parallel.fsdp import FSDP, size_based_auto_wrap_policy, transformer_auto_wrap_policy

    policy = {"layer": transformer_auto_wrap_policy({TransformerEncoderLayer}),
              "leaf": size_based_auto_wrap_policy(500)}[policy_kind]
    m = FSDP(_make_model(layers=layers), auto_wrap_policy=policy, device_id=torch.device("cpu"),
             sharding_strategy="FULL_SHARD", ring=ring)
    if ring:
        for r in m._rings.values():
            for b in r.bufs:
                b.fill_(float("nan"))
    opt = torch.optim.SGD(m.parameters(), lr=1e-1, momentum=0.9)
    per = 8 // world
    for s in range(steps):
        x, y = _batch(s)
        x, y = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
        h = per // 2
        for xx, yy in ((x[:h], y[:h]), (x[h:], y[h:])):
            (m.forward_loss(xx, yy, ignore_index=-100) / 2).backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
    return {"sd": m.full_state_dict(rank0_only=True), "ring": m.ring}


@pytest.mark.parametrize("ring", [2, 3])
def test_fsdp_ring_world1_accumulates_like_non_ring(ring):
    """World 1 identity ring path with .grad already present (accumulation, set_to_none=False):
    equal to the non-ring wrapper doing the same thing (the r05 bug doubled the latest gradient)."""
    base = run_world(_fsdp_accum_train, 1, (0,))[0]["sd"]
    got = run_world(_fsdp_accum_train, 1, (ring,))[0]
    assert got["ring"] == ring
    for k in base:
        torch.testing.assert_close(got["sd"][k], base[k], rtol=1e-5, atol=1e-6, msg=k)


@pytest.mark.parametrize("world", [1, 2])
@pytest.mark.parametrize("ring", [2, 3])
def test_fsdp_ring_nested_units_match_single_process(world, ring):
    """Size-based wrapping nests units (the attention module holds its wrapped out-projection):
    a nested unit never shares a ring slot with an ancestor, so the NaN-poisoned ring still
    trains exactly like the non-ring wrapper."""
    base = run_world(_fsdp_accum_train, world, (0, "leaf", 2))[0]["sd"]
    got = run_world(_fsdp_accum_train, world, (ring, "leaf", 2))[0]
    assert got["ring"] == ring
    for k in base:
        torch.testing.assert_close(got["sd"][k], base[k], rtol=1e-4, atol=1e-5, msg=k)


def test_fsdp_ring_slot_assignment_rules():
    import torch.nn as nn

    from hyperion.parallel.fsdp import FSDP

    class Box(nn.Module):
        def __init__(self, inner):
            super().__init__()
            self.inner = inner
            self.w = nn.Linear(4, 4)

    flat = nn.Sequential(*[nn.Linear(4, 4) for _ in range(5)])
    assert FSDP._ring_slots(flat, list(flat), 3) == [0, 1, 2, 0, 1]
    # Box(Box(Linear)): three nested units -> each in its own slot; needs 3 slots
    leaf = nn.Linear(4, 4)
    mid = Box(leaf)
    top = Box(mid)
    root = nn.Sequential(top)
    units = [leaf, mid, top]  # post-order
    slots = FSDP._ring_slots(root, units, 3)
    assert len(set(slots)) == 3
    assert FSDP._ring_slots(root, units, 2) is None  # nesting depth 3 > 2 slots
    m = FSDP(root, auto_wrap_policy=lambda mod, n: isinstance(mod, (nn.Linear, Box)) and mod is not top.w
             and mod is not mid.w, device_id=torch.device("cpu"), ring=2)
    assert m.ring == 0  # fell back to reshard-after-forward
