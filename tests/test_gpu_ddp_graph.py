"""Captured data-parallel step (fwd+bwd graph(s), bucket all-reduces between replays, optimizer
graph) on one GPU.

* single rank, bucket machinery forced on: after ONE captured replay the reduced bucket
  gradients equal the eager gradients at the same weights (tight tolerance — a skipped bucket,
  an all-zero bottom stage or a bucket overwritten while reduced would fail), and the step
  matches an eager reference;
* two gloo ranks on the same GPU (the 8-GPU path rehearsed with real inter-process collectives):
  after several captured three-graph steps both ranks hold bit-identical parameters, equal to
  the eager ``split_step`` schedule run from the same start.
"""
import copy
import os
import socket

import pytest
import torch

from dist_utils import run_world
from parity import assert_losses_match, assert_update_parity, snapshot

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make(seed=0):
    from hyperion.models.resnet import resnet18
    from hyperion.train.amp import cast_for_compute

    torch.manual_seed(seed)
    m = resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    return m


def _pin_deterministic():
    # MIOpen's default stem-conv wgrad algorithm is not bitwise deterministic: pin it so the
    # comparisons check the DDP schedule, not last-bit noise
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    return prev


def _replay_grads_only(step, ddp):
    """Replay the captured fwd+bwd graph(s) and the all-reduces, but not the optimizer graph."""
    step.graph.replay()
    if step.graph3 is not None:
        works = ddp.allreduce_buckets(step._phase1, wait=False)
        step.graph2.replay()
        works += ddp.allreduce_buckets(step._phase2, wait=False)
        for w in works:
            w.wait()
    else:
        ddp.allreduce_buckets()
    torch.cuda.synchronize()


@pytest.mark.parametrize("split,native", [(False, False), (True, False), (True, True)])
def test_ddp_graph_step_grads_match_eager(split, native):
    """split: three graphs (top fwd+bwd | bottom bwd | optimizer) with the top buckets' all-reduce
    issued between graphs 1 and 2 without a stream wait; native: Hyperion's RCCL communicator
    (single rank) instead of the torch.distributed no-op comm."""
    import torch.distributed as dist

    from hyperion.ops.optim import FusedAdam, grad_of
    from hyperion.parallel import DDP
    from hyperion.train.step import TrainStep

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    prev = _pin_deterministic()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        x = torch.rand(16, 3, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = torch.rand(16, 10, device="cuda")
        comm = None
        if native:
            from hyperion.parallel.comm import NativeComm

            comm = NativeComm(torch.device("cuda", 0))
        ddp = DDP(_make(), bucket_cap_mb=2.0, first_bucket_mb=0.5, broadcast_buffers=False, buckets_at_world_1=True,
                  comm=comm)
        assert ddp.bucketed and len(ddp.bucket_sizes()) > 1
        assert {b.buf.dtype for b in ddp._buckets} == {torch.float32}  # fp32 reduction by default
        dopt = FusedAdam(ddp.parameters(), lr=1e-3, zero_grad_in_step=True)
        dstep = TrainStep(ddp, dopt, torch.nn.MSELoss(), amp_dtype=None, graph=True, warmup_iters=2,
                          split_backward=split, ddp_schedule="split3")
        dstep(x, y)  # warm-up + capture + one replay (weights move)
        assert dstep.graph2 is not None and (dstep.graph3 is not None) == split
        if split:
            assert dstep._phase1 and dstep._phase2  # both halves own buckets

        # reference at the SAME weights, eager
        ref = _make()
        ref.load_state_dict(ddp.module.state_dict())
        out = ref(x)
        rloss = torch.nn.functional.mse_loss(out.float(), y)
        rloss.backward()

        _replay_grads_only(dstep, ddp)
        torch.testing.assert_close(dstep.static_loss.float(), rloss.detach().float(), rtol=1e-3, atol=1e-6)
        n_main = 0
        for (n, rp), dp in zip(ref.named_parameters(), ddp.module.parameters()):
            g = grad_of(dp)
            assert g is not None and g.abs().sum() > 0, n  # every bucket (top AND bottom stage) filled
            n_main += int(getattr(dp, "main_grad", None) is not None)
            torch.testing.assert_close(g.float(), rp.grad.float(), rtol=1e-3, atol=1e-5, msg=n)
        assert n_main > 0  # bf16 conv / fc weights read fp32 main_grads

        # and the optimizer graph applies exactly the update of those gradients
        before = {n: p.detach().float().clone() for n, p in ddp.module.named_parameters()}
        dstep.graph3.replay() if dstep.graph3 is not None else dstep.graph2.replay()
        torch.cuda.synchronize()
        moved = sum(int(not torch.equal(before[n], p.detach().float())) for n, p in ddp.module.named_parameters())
        assert moved > 0.9 * len(before)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
        dist.destroy_process_group()


def _two_rank_graph(rank, world, steps, schedule="split3"):
    os.environ["HYPERION_COMM"] = "torch"  # gloo collectives between the two processes
    torch.cuda.set_device(0)
    _pin_deterministic()
    from hyperion.ops.optim import FusedAdam
    from hyperion.parallel import DDP
    from hyperion.train.step import TrainStep

    g = torch.Generator(device="cuda").manual_seed(100 + rank)
    xs = [torch.rand(8, 3, 32, 32, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
          for _ in range(steps)]
    ys = [torch.rand(8, 10, device="cuda", generator=g) for _ in range(steps)]
    res = {}
    for mode in ("graph", "split_step"):
        ddp = DDP(_make(seed=rank), bucket_cap_mb=2.0, first_bucket_mb=0.5, broadcast_buffers=False)
        before = snapshot(ddp.module.named_parameters())
        opt = FusedAdam(ddp.parameters(), lr=1e-3, zero_grad_in_step=True)
        losses = []
        if mode == "graph":
            st = TrainStep(ddp, opt, torch.nn.MSELoss(), amp_dtype=None, graph=True, warmup_iters=1,
                           ddp_schedule=schedule)
            losses.append(float(st(xs[0], ys[0])))  # warm-up step + capture + replay: step 0 twice
            for i in range(1, steps):
                losses.append(float(st(xs[i], ys[i])))
            graphs = st.graph3 is not None if schedule == "split3" else st.seg is not None
        else:
            ddp.defer_allreduce = True
            st = TrainStep(ddp, opt, torch.nn.MSELoss(), amp_dtype=None, graph=False)
            st.split_step(xs[0], ys[0])  # mirror the warm-up step
            for i in range(steps):
                losses.append(float(st.split_step(xs[i], ys[i])))
            graphs = None
        torch.cuda.synchronize()
        res[mode] = {"params": [p.detach().float().cpu() for p in ddp.module.parameters()], "graph3": graphs,
                     "before": before, "after": snapshot(ddp.module.named_parameters()), "losses": losses}
    return res


@pytest.mark.parametrize("schedule", ["split3", "segmented"])
def test_two_rank_gloo_graph_step_replicas_identical(schedule):
    """auto: the three-graph split; segmented: bench.py's N>1 default (graph segments with the
    bucket all-reduces as eager holes)."""
    res = run_world(_two_rank_graph, 2, (4, schedule), timeout=600)
    assert res[0]["graph"]["graph3"] and res[1]["graph"]["graph3"]
    for a, b in zip(res[0]["graph"]["params"], res[1]["graph"]["params"]):
        assert torch.equal(a, b)  # replicas bit-identical after captured steps
    for r in (0, 1):  # same schedule, eager: per-step losses and the parameter UPDATE (tests/parity.py)
        g, e = res[r]["graph"], res[r]["split_step"]
        assert all(torch.equal(g["before"][k], e["before"][k]) for k in g["before"])
        assert_losses_match(g["losses"], e["losses"], rtol=1e-2, what=f"rank {r}")
        assert_update_parity(e["before"], g["after"], e["after"], rel=2e-2, what=f"rank {r}")


@pytest.mark.parametrize("native,schedule", [(False, "segmented"), (True, "segmented"), (True, "graph")])
def test_ddp_segmented_schedule_matches_eager(native, schedule):
    """``TrainStep(ddp_schedule="segmented")``: the whole step captured as graph segments with the
    bucket all-reduces as eager holes (bench.py --ddp-schedule segmented).  Per-step losses and the
    parameter update over 4 steps equal the eager DDP step from the same start."""
    import torch.distributed as dist

    from hyperion.ops.optim import FusedAdam
    from hyperion.parallel import DDP
    from hyperion.train.step import TrainStep

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    prev = _pin_deterministic()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        g = torch.Generator(device="cuda").manual_seed(3)
        xs = [torch.rand(16, 3, 32, 32, device="cuda", generator=g).bfloat16().contiguous(
            memory_format=torch.channels_last) for _ in range(4)]
        ys = [torch.rand(16, 10, device="cuda", generator=g) for _ in range(4)]
        res = {}
        for mode in ("segmented", "eager"):
            comm = None
            if native:
                from hyperion.parallel.comm import NativeComm

                comm = NativeComm(torch.device("cuda", 0))
            ddp = DDP(_make(), bucket_cap_mb=2.0, first_bucket_mb=0.5, broadcast_buffers=False,
                      buckets_at_world_1=True, comm=comm)
            before = snapshot(ddp.module.named_parameters())
            opt = FusedAdam(ddp.parameters(), lr=1e-3, zero_grad_in_step=mode == "segmented")
            st = TrainStep(ddp, opt, torch.nn.MSELoss(), amp_dtype=None, graph=mode == "segmented",
                           warmup_iters=1, ddp_schedule=schedule)
            losses = [float(st(xs[0], ys[0]))]  # graph mode: warm-up step + capture + replay = step 0 twice
            if mode == "eager":
                losses = [float(st(xs[0], ys[0]))]
            for i in range(1, 4):
                losses.append(float(st(xs[i], ys[i])))
            torch.cuda.synchronize()
            if mode == "segmented" and schedule == "segmented":
                # an issue and a wait hole per bucket (adjacent holes share one replayed segment boundary)
                assert st.seg is not None and st.seg.num_holes >= len(ddp.bucket_sizes()) and st.seg.num_segments > 1
            elif mode == "segmented":  # ONE graph, the RCCL all-reduces recorded into it
                assert st.seg is None and st.graph is not None and st.graph2 is None
            res[mode] = (before, snapshot(ddp.module.named_parameters()), losses)
        (b0, a_seg, l_seg), (b1, a_eag, l_eag) = res["segmented"], res["eager"]
        assert all(torch.equal(b0[k], b1[k]) for k in b0)
        assert_losses_match(l_seg, l_eag, rtol=1e-2, what="segmented vs eager")
        assert_update_parity(b1, a_seg, a_eag, rel=2e-2, what="segmented vs eager")
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
        dist.destroy_process_group()
