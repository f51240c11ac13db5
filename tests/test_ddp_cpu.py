"""Hyperion DDP on gloo: bucketed all-reduce parity with single-process training, no_sync, buffers."""
import torch

from dist_utils import run_world


def _model(seed=0):
    from hyperion.models.resnet import resnet18

    torch.manual_seed(seed)
    return resnet18(num_classes=10)


def _data(step, n=8):
    g = torch.Generator().manual_seed(50 + step)
    return torch.randn(n, 3, 32, 32, generator=g), torch.randint(0, 10, (n,), generator=g)


def _ref(steps):
    m = _model()
    m.train()
    opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
    for s in range(steps):
        x, y = _data(s)
        # DDP semantics: per-rank BN statistics; emulate by splitting the batch into two halves
        loss = sum(torch.nn.functional.cross_entropy(m(xx), yy) for xx, yy in ((x[:4], y[:4]), (x[4:], y[4:]))) / 2
        loss.backward()
        opt.step()
        opt.zero_grad()
    return {k: v for k, v in m.state_dict().items() if "running" not in k and "num_batches" not in k}


def _ddp(rank, world, steps, bucket_mb):
    from hyperion.parallel import DDP

    m = DDP(_model(seed=rank), bucket_cap_mb=bucket_mb, first_bucket_mb=0.1, broadcast_buffers=False)
    opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
    for s in range(steps):
        x, y = _data(s)
        x, y = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
    sd = {k: v for k, v in m.state_dict().items() if "running" not in k and "num_batches" not in k}
    return {"sd": sd, "buckets": m.bucket_sizes()}


def test_ddp_matches_single_process_and_ranks_agree():
    ref = _ref(3)
    res = run_world(_ddp, 2, (3, 1.0))
    assert len(res[0]["buckets"]) > 3
    for k in ref:
        torch.testing.assert_close(res[0]["sd"][k], res[1]["sd"][k], rtol=0, atol=0, msg=k)
        torch.testing.assert_close(res[0]["sd"][k], ref[k], rtol=1e-4, atol=1e-5, msg=k)


def _ddp_no_sync(rank, world):
    from hyperion.parallel import DDP

    m = DDP(_model(), bucket_cap_mb=4.0)
    x, y = _data(0)
    with m.no_sync():
        torch.nn.functional.cross_entropy(m(x[rank::2]), y[rank::2]).backward()
    local = [p.grad.clone() for p in m.parameters()]
    return local[0].sum().item()


def test_ddp_no_sync_keeps_local_grads():
    res = run_world(_ddp_no_sync, 2)
    assert res[0] != res[1]


def _ddp_deferred(rank, world, steps):
    """defer_allreduce: backward packs buckets only; allreduce_buckets() between backward and step."""
    from hyperion.parallel import DDP

    m = DDP(_model(seed=rank), bucket_cap_mb=1.0, first_bucket_mb=0.1, broadcast_buffers=False)
    m.defer_allreduce = True
    opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
    for s in range(steps):
        x, y = _data(s)
        x, y = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
        torch.nn.functional.cross_entropy(m(x), y).backward()
        m.allreduce_buckets()
        opt.step()
        opt.zero_grad(set_to_none=False)  # graph-style: gradients keep their bucket addresses
    return {k: v for k, v in m.state_dict().items() if "running" not in k and "num_batches" not in k}


def test_ddp_deferred_allreduce_matches_single_process():
    ref = _ref(3)
    res = run_world(_ddp_deferred, 2, (3,))
    for k in ref:
        torch.testing.assert_close(res[0][k], res[1][k], rtol=0, atol=0, msg=k)
        torch.testing.assert_close(res[0][k], ref[k], rtol=1e-4, atol=1e-5, msg=k)


def _ddp_split(rank, world, steps):
    """TrainStep.split_step: top-stage backward, its complete buckets all-reduced without waiting
    while the bottom-stage backward runs, then the rest (the captured 3-graph schedule, eager)."""
    from hyperion.parallel import DDP
    from hyperion.train.step import TrainStep

    m = DDP(_model(seed=rank), bucket_cap_mb=1.0, first_bucket_mb=0.1, broadcast_buffers=False)
    m.defer_allreduce = True
    opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
    step = TrainStep(m, opt, torch.nn.functional.cross_entropy, amp_dtype=None, graph=False)
    calls = []
    orig = m.allreduce_buckets

    def spy(indices=None, wait=True):
        calls.append(list(indices))
        return orig(indices, wait)

    m.allreduce_buckets = spy
    firsts = []
    for s in range(steps):
        x, y = _data(s)
        x, y = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
        step.split_step(x, y)
        firsts.append(m.complete_buckets())  # state reset after the full backward: []
    sd = {k: v for k, v in m.state_dict().items() if "running" not in k and "num_batches" not in k}
    stage = {id(p): i for i, mods in enumerate(m.module.graph_stage_modules()) for mod in mods
             for p in mod.parameters()}
    straddle = [b.index for b in m._buckets if len({stage[id(p)] for p in b.params}) != 1]
    return {"sd": sd, "firsts": firsts, "n": len(m.bucket_sizes()), "calls": calls, "straddle": straddle}


def test_ddp_split_backward_overlap_matches_single_process():
    ref = _ref(3)
    res = run_world(_ddp_split, 2, (3,))
    assert res[0]["n"] > 3 and all(f == [] for f in res[0]["firsts"])
    first, rest = res[0]["calls"][0], res[0]["calls"][1]
    assert first and rest and sorted(first + rest) == list(range(res[0]["n"]))  # a real two-phase split
    assert res[0]["calls"] == res[1]["calls"] and res[0]["straddle"] == []
    for k in ref:
        torch.testing.assert_close(res[0]["sd"][k], res[1]["sd"][k], rtol=0, atol=0, msg=k)
        torch.testing.assert_close(res[0]["sd"][k], ref[k], rtol=1e-4, atol=1e-5, msg=k)


def _ddp_lowp(rank, world, comm_dtype):
    """bf16 compute copies: the reduced gradient is the fp32 average of the ranks' bf16 gradients
    (fp32 buckets, ``main_grad``) or its bf16 rounding (opt-in bf16 buckets, ``grad``)."""
    import copy

    import torch.distributed as dist

    from hyperion.ops.optim import FusedAdam, grad_of
    from hyperion.parallel import DDP
    from hyperion.train.amp import cast_for_compute

    base = cast_for_compute(_model(seed=0), torch.bfloat16)
    plain = copy.deepcopy(base)
    x, y = _data(0)
    x, y = x[rank * 4:(rank + 1) * 4].to(torch.bfloat16), y[rank * 4:(rank + 1) * 4]
    torch.nn.functional.cross_entropy(plain(x).float(), y).backward()
    local = [p.grad.float() for p in plain.parameters()]
    gathered = []
    for g in local:
        out = [torch.empty_like(g) for _ in range(world)]
        dist.all_gather(out, g)
        gathered.append(sum(out) / world)
    m = DDP(base, bucket_cap_mb=1.0, first_bucket_mb=0.1, broadcast_buffers=False, comm_dtype=comm_dtype)
    torch.nn.functional.cross_entropy(m(x).float(), y).backward()
    got = [grad_of(p) for p in m.parameters()]
    dtypes = sorted({str(g.dtype) for g in got})
    err = max(float((g.float() - e).abs().max()) for g, e in zip(got, gathered))
    err_bf16 = max(float((g.float() - e.to(torch.bfloat16).float()).abs().max()) for g, e in zip(got, gathered))
    has_main = any(getattr(p, "main_grad", None) is not None for p in m.parameters())
    opt = FusedAdam(m.parameters(), lr=1e-3)
    opt.step()
    return {"err": err, "err_bf16": err_bf16, "dtypes": dtypes, "has_main": has_main,
            "params": [p.detach().float().clone() for p in m.parameters()]}


def test_ddp_bf16_compute_reduces_in_fp32_by_default():
    res = run_world(_ddp_lowp, 2, (torch.float32,))
    for r in (0, 1):
        assert res[r]["has_main"] and "torch.float32" in res[r]["dtypes"]
        assert res[r]["err"] == 0.0  # exactly the fp32 average of the bf16 rank gradients
    for a, b in zip(res[0]["params"], res[1]["params"]):
        torch.testing.assert_close(a, b, rtol=0, atol=0)


def test_ddp_bf16_buckets_opt_in():
    res = run_world(_ddp_lowp, 2, (torch.bfloat16,))
    for r in (0, 1):
        assert res[r]["dtypes"] == ["torch.bfloat16"]  # every bucket on the wire in bf16
        assert res[r]["err_bf16"] <= 1e-2  # gloo's bf16 sum: one rounding of the fp32 average
    for a, b in zip(res[0]["params"], res[1]["params"]):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
