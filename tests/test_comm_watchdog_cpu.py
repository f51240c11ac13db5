"""Native communicator watchdog (csrc/comm/watchdog.h) on the CPU via the WatchdogSim harness:
the SAME C++ Watchdog class the RCCL communicator uses, with simulated work handles.

Reference: collectives run under a process-group timeout (02_development/distributed_utils.py:106-111,
test_nccl.py:26-29); the native comm path must fail instead of hanging."""
import time

import pytest

from hyperion.ops import _native

pytestmark = pytest.mark.skipif(not _native.available(), reason="hyperion._C not built")


def _sim(timeout_s=0.2, poll_ms=1.0):
    return _native.native().WatchdogSim(timeout_s, poll_ms)


def test_completed_work_retires_without_failure():
    w = _sim(timeout_s=0.5)
    ids = [w.submit(f"all_reduce #{i}") for i in range(5)]
    for i in ids:
        w.complete(i)
    assert w.drain(2.0)
    assert not w.failed() and w.error() == "" and w.aborts() == 0 and w.pending() == 0


def test_deadline_expiry_fails_once_and_names_the_collective():
    w = _sim(timeout_s=0.1)
    a = w.submit("all_reduce #1 (4096 B, rank 0/2)")
    w.complete(a)
    w.submit("reduce_scatter #2 (8 B, rank 0/2)")  # never completes: a dead peer
    t0 = time.monotonic()
    while not w.failed() and time.monotonic() - t0 < 5.0:
        time.sleep(0.005)
    took = time.monotonic() - t0
    assert w.failed()
    assert 0.05 < took < 2.0
    assert "reduce_scatter #2" in w.error() and "timeout" in w.error()
    time.sleep(0.05)
    assert w.aborts() == 1  # the failure action (ncclCommAbort in production) runs exactly once
    assert w.pending() == 0
    assert not w.drain(0.1)


def test_head_of_line_decides_deadline():
    # collectives on one stream retire in order: a completed LATER op must not hide a stuck head
    w = _sim(timeout_s=0.1)
    a = w.submit("head")
    b = w.submit("tail")
    w.complete(b)
    time.sleep(0.3)
    assert w.failed() and "'head'" in w.error()
    assert a == 0


def test_async_error_fails_pending_and_idle():
    w = _sim(timeout_s=30.0)
    w.submit("all_gather #1")
    w.set_async_error("remote process exited or there was a network error")
    t0 = time.monotonic()
    while not w.failed() and time.monotonic() - t0 < 5.0:
        time.sleep(0.005)
    assert w.failed() and "async error" in w.error() and "network error" in w.error()


def test_device_side_failure_probe():
    w = _sim(timeout_s=30.0)
    i = w.submit("broadcast #7")
    w.fail_op(i)
    t0 = time.monotonic()
    while not w.failed() and time.monotonic() - t0 < 5.0:
        time.sleep(0.005)
    assert "broadcast #7" in w.error() and "failed on the device" in w.error()


def test_fault_spec_stall_parses_and_targets_one_collective(monkeypatch):
    from hyperion.utils.fault import comm_stall_s, maybe_inject, parse

    assert parse("1:3:stall") == (1, 3, "stall")
    monkeypatch.setenv("HYPERION_FAULT_STALL_S", "2.5")
    assert comm_stall_s(1, 3, "1:3:stall") == 2.5
    assert comm_stall_s(0, 3, "1:3:stall") == 0.0
    assert comm_stall_s(1, 2, "1:3:stall") == 0.0
    assert maybe_inject(1, 3, "1:3:stall") is False  # a comm fault, not a trainer-step fault


def test_group_key_is_per_group(monkeypatch):
    from hyperion.parallel.comm import group_key

    assert group_key(None) == "local"  # no process group initialised in this test process
