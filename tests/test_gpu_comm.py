"""Native RCCL communicator (csrc/comm/rccl_comm.cpp) on one GPU (world 1: every collective is an
identity, which still exercises the bootstrap, the comm stream, event fencing and recordStream)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture()
def pg():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


def test_native_comm_collectives_world1(pg):
    from hyperion.ops import _native
    from hyperion.parallel.comm import NativeComm

    assert _native.native().rccl_version() > 0
    c = NativeComm(torch.device("cuda", 0))
    x = torch.arange(1024, device="cuda", dtype=torch.float32)
    w = c.all_reduce(x, "sum")
    w.wait()
    torch.testing.assert_close(x, torch.arange(1024, device="cuda", dtype=torch.float32))
    out = torch.empty(1024, device="cuda", dtype=torch.bfloat16)
    c.all_gather(out, x.to(torch.bfloat16)).wait()
    torch.testing.assert_close(out.float(), x.to(torch.bfloat16).float())
    rs = torch.empty(1024, device="cuda")
    c.reduce_scatter(rs, x, "sum").wait()
    torch.testing.assert_close(rs, x)
    a2a = torch.empty_like(x)
    c.all_to_all(a2a, x).wait()
    torch.testing.assert_close(a2a, x)
    ts = [torch.ones(10, device="cuda"), torch.full((7,), 2.0, device="cuda")]
    c.all_reduce_coalesced(ts, "sum").synchronize()
    assert ts[1].sum().item() == 14.0
    c.barrier()
    assert c.async_error() == ""
    c.destroy()


@pytest.mark.parametrize("dt,n", [(torch.bfloat16, 132480), (torch.bfloat16, 131392), (torch.bfloat16, 133568),
                                  (torch.float32, 16704), (torch.float32, 17024)])
def test_native_comm_avg_writes_every_element(pg, dt, n):
    """"avg" reductions run as SUM + 1/world on the comm stream: RCCL's own ncclAvg (torch-bundled
    2.26.6) left the last 4-16 outputs of these reduce-scatter sizes unwritten (an FSDP unit's
    flat gradient tail — its last LayerNorm bias — came back stale)."""
    from hyperion.parallel.comm import NativeComm

    c = NativeComm(torch.device("cuda", 0))
    x = torch.randn(n, device="cuda").to(dt)
    out = torch.full((n,), 7.0, device="cuda", dtype=dt)
    c.reduce_scatter(out, x, "avg").wait()
    torch.testing.assert_close(out, x, rtol=0, atol=0)
    y = x.clone()
    c.all_reduce(y, "avg").wait()
    torch.testing.assert_close(y, x, rtol=0, atol=0)
    c.destroy()


@pytest.mark.parametrize("div", [2, 8])
def test_native_comm_avg_scale_path_world_gt_1(pg, div):
    """The world > 1 branch of RcclComm::scale_avg (SUM, then x 1/world on the comm stream before
    the completion event) on one GPU: the divisor is forced to ``div`` while RCCL reduces over one
    rank, so the result must be exactly x / div — and visible to the compute stream after wait()
    without any host synchronisation (a consumer kernel reads it at once)."""
    from hyperion.parallel.comm import NativeComm

    c = NativeComm(torch.device("cuda", 0))
    c._c.set_avg_divisor(div)
    x = torch.randn(1 << 20, device="cuda")
    y = x.clone()
    c.all_reduce(y, "avg").wait()
    got = y * 1.0  # compute-stream consumer right after the wait
    torch.testing.assert_close(got, x / div, rtol=0, atol=0)
    out = torch.full((4099,), 3.0, device="cuda", dtype=torch.bfloat16)
    xb = torch.randn(4099, device="cuda").to(torch.bfloat16)
    c.reduce_scatter(out, xb, "avg").wait()
    torch.testing.assert_close(out, xb * (1.0 / div), rtol=0, atol=0)
    ts = [torch.ones(10, device="cuda"), torch.full((7,), 2.0, device="cuda")]
    c.all_reduce_coalesced(ts, "avg").wait()
    torch.testing.assert_close(ts[1], torch.full((7,), 2.0 / div, device="cuda"))
    y2 = x.clone()
    c.all_reduce(y2, "sum").wait()  # "sum" is never scaled
    torch.testing.assert_close(y2, x, rtol=0, atol=0)
    c._c.set_avg_divisor(0)
    c.destroy()


def test_native_comm_orders_against_compute_stream(pg):
    # a producer kernel on the current stream, then the collective on the comm stream, then a
    # consumer: the result must see the producer's data and the consumer must see the collective
    from hyperion.parallel.comm import NativeComm

    c = NativeComm(torch.device("cuda", 0))
    x = torch.zeros(1 << 22, device="cuda")
    for _ in range(20):
        x.add_(1.0)  # queue work on the compute stream
    w = c.all_reduce(x, "sum")
    w.wait()
    y = x * 2
    torch.cuda.synchronize()
    assert float(y[0]) == 40.0 and float(y[-1]) == 40.0
    c.destroy()


def test_native_comm_watchdog_times_out_stalled_collective(pg, monkeypatch):
    """A device-side stall on the comm stream (HYPERION_FAULT=0:2:stall) makes the 2nd collective
    miss a 0.5 s deadline: the watchdog aborts the communicator and the next wait() raises a clean
    RuntimeError naming the collective, instead of hanging."""
    import time

    from hyperion.parallel.comm import NativeComm

    monkeypatch.setenv("HYPERION_FAULT", "0:2:stall")
    monkeypatch.setenv("HYPERION_FAULT_STALL_S", "3")
    c = NativeComm(torch.device("cuda", 0), timeout_s=0.5)
    x = torch.ones(256, device="cuda")
    c.all_reduce(x, "sum").wait()  # seq 1: healthy
    torch.cuda.synchronize()
    assert c.error() == ""
    t0 = time.monotonic()
    w = c.all_reduce(x, "sum")  # seq 2: its comm stream sleeps ~3 s first
    while c.error() == "" and time.monotonic() - t0 < 20.0:
        time.sleep(0.01)
    took = time.monotonic() - t0
    assert "all_reduce #2" in c.error() and "timeout" in c.error(), c.error()
    assert took < 2.9, took  # detected at the deadline, not after the stall drained
    with pytest.raises(RuntimeError, match="all_reduce #2"):
        w.wait()
    with pytest.raises(RuntimeError, match="communicator failed"):
        c.all_reduce(x, "sum")
    torch.cuda.synchronize()  # the stall kernel drains; the device stays usable
    assert float((x * 2).sum()) == 512.0
    c.destroy()
