"""Captured FSDP steps (train/segments.py): the step recorded once as graph segments with the
all-gathers / reduce-scatters / clip all-reduce as eager holes between them.

* one rank: persistent FSDP over the LM (GPT-2-style layers, one unit per layer), captured steps
  match eager steps from the same start (the captured schedule replays the same kernels);
* two gloo ranks on one GPU (the multi-GPU schedule rehearsed with real inter-process
  collectives): captured steps leave both ranks with the same gathered parameters, equal to the
  eager FSDP schedule run from the same start.

Reference: torch FSDP FULL_SHARD trainers, eager every step (02_development/distributed_utils.py:318-354).
"""
import os

import pytest
import torch

from dist_utils import run_world
from parity import assert_losses_match, assert_update_parity

pytestmark = pytest.mark.gpu


def _lm(seed=0, layers=2):
    from hyperion.models.simple_lm import SimpleTransformerLM

    torch.manual_seed(seed)
    return SimpleTransformerLM(vocab_size=512, emb_dim=128, n_heads=2, n_layers=layers, ff_dim=256, dropout=0.0,
                               causal=True).cuda()


def _fsdp_run(steps, graphed, seed=0, rank=0, coll=False, ring=0, layers=2):
    from hyperion.models.transformer import TransformerEncoderLayer
    from hyperion.ops.optim import FusedAdam
    from hyperion.parallel.fsdp import FSDP, MixedPrecision, transformer_auto_wrap_policy
    from hyperion.train.segments import SegmentedStep

    bf = torch.bfloat16
    m = FSDP(_lm(seed, layers), auto_wrap_policy=transformer_auto_wrap_policy({TransformerEncoderLayer}),
             device_id=torch.device("cuda", 0), mixed_precision=MixedPrecision(bf, bf, bf), persistent=not ring,
             collectives_at_world_1=coll, ring=ring)
    opt = FusedAdam(list(m.parameters()), lr=1e-3, weight_decay=0.01, adamw=True)
    g = torch.Generator(device="cuda").manual_seed(7 + rank)
    data = [torch.randint(0, 512, (4, 33), device="cuda", generator=g) for _ in range(steps)]
    ids = data[0].clone()
    before = {k: v.double() for k, v in m.full_state_dict(rank0_only=False, offload_to_cpu=True).items()}

    def body():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=bf):
            loss = m.forward_loss(ids[:, :-1], ids[:, 1:])
        loss.backward()
        m.clip_grad_norm_(1.0)
        opt.step()
        return loss.detach()

    losses = []
    if graphed:
        st = SegmentedStep(body, warmup=1, module=m)
        for i in range(steps):
            ids.copy_(data[i])
            if i == 0:
                body()  # mirror the single warm-up call below so both schedules take steps+1 steps
            losses.append(float(st()))
        nseg = st.seg.num_segments
    else:
        for i in range(steps):
            ids.copy_(data[i])
            if i == 0:
                body()
                body()  # SegmentedStep: one warm-up call + the capture pass are steps too
            losses.append(float(body()))
        nseg = 0
    torch.cuda.synchronize()
    full = m.full_state_dict(rank0_only=False, offload_to_cpu=True)
    return {"losses": losses, "params": {k: v.float() for k, v in full.items()}, "before": before, "segments": nseg,
            "comm": type(m.comm).__name__, "identity": m.identity}


def test_fsdp_segmented_capture_matches_eager_one_rank():
    os.environ["HYPERION_COMM"] = "torch"
    a = _fsdp_run(4, graphed=True)
    b = _fsdp_run(4, graphed=False)
    assert a["segments"] >= 1
    _parity(a, b)


def _parity(a, b, what=""):
    """Captured vs eager from the same start: per-step losses and the parameter UPDATE (not the
    parameters, whose ~1e-3 total movement hides a skipped or stale step; tests/parity.py)."""
    for k in b["before"]:
        assert torch.equal(a["before"][k], b["before"][k]), k  # the same starting point
    assert_losses_match(a["losses"], b["losses"], what=what)
    assert_update_parity(b["before"], a["params"], b["params"], rel=2e-2, what=what)


def test_fsdp_native_collectives_at_world_1_segmented_matches_eager():
    """collectives_at_world_1: the gathers / reduce-scatters run over the native RCCL communicator
    on one GPU (a real collective, not the identity copy) inside the segmented capture, and the
    captured steps match the eager identity schedule."""
    import socket

    import torch.distributed as dist

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    os.environ["HYPERION_COMM"] = "native"
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        a = _fsdp_run(4, graphed=True, coll=True)
        b = _fsdp_run(4, graphed=False)
    finally:
        dist.destroy_process_group()
        os.environ["HYPERION_COMM"] = "torch"
    assert a["comm"] == "NativeComm" and not a["identity"] and b["identity"]
    assert a["segments"] > 1  # the RCCL collectives are eager holes between captured segments
    _parity(a, b, "native collectives")


def _two_rank(rank, world, steps, ring=0, layers=2):
    os.environ["HYPERION_COMM"] = "torch"  # gloo collectives between the two processes
    torch.cuda.set_device(0)
    return {"graph": _fsdp_run(steps, True, rank=rank, ring=ring, layers=layers),
            "eager": _fsdp_run(steps, False, rank=rank, ring=ring, layers=layers)}


def test_fsdp_segmented_capture_two_gloo_ranks():
    res = run_world(_two_rank, 2, (3,), timeout=600)
    g0, g1 = res[0]["graph"], res[1]["graph"]
    assert g0["segments"] > 1 and g1["segments"] > 1  # collectives became holes between segments
    for k in g0["params"]:
        assert torch.equal(g0["params"][k], g1["params"][k])  # one set of gathered params on both ranks
    for r in (0, 1):
        _parity(res[r]["graph"], res[r]["eager"], f"rank {r}")


def test_fsdp_ring_native_collectives_segmented_matches_eager():
    """FULL_SHARD ring (2 fixed-address slots for 4 layer units, evicting each other every step)
    captured as graph segments with real RCCL gathers / reduce-scatters at world 1: the captured
    steps match the eager identity schedule, and the ring keeps 2 units' buffers, not 4."""
    import socket

    import torch.distributed as dist

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    os.environ["HYPERION_COMM"] = "native"
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        a = _fsdp_run(4, graphed=True, coll=True, ring=2, layers=4)
        b = _fsdp_run(4, graphed=False, layers=4)
    finally:
        dist.destroy_process_group()
        os.environ["HYPERION_COMM"] = "torch"
    assert a["comm"] == "NativeComm" and not a["identity"]
    assert a["segments"] > 1
    _parity(a, b, "ring native collectives")


def test_fsdp_ring_segmented_capture_two_gloo_ranks():
    res = run_world(_two_rank, 2, (3, 2, 4), timeout=600)
    g0, g1 = res[0]["graph"], res[1]["graph"]
    for k in g0["params"]:
        assert torch.equal(g0["params"][k], g1["params"][k])
    for r in (0, 1):
        _parity(res[r]["graph"], res[r]["eager"], f"ring rank {r}")
