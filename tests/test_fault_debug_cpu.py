"""Failure detection and consistency checks on gloo."""
import os
import subprocess
import sys
import time

import pytest
import torch

from dist_utils import free_port, run_world

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fault_spec_parsing():
    from hyperion.utils.fault import maybe_inject, parse

    assert parse("1:5:exit") == (1, 5, "exit")
    assert parse("") is None
    with pytest.raises(ValueError):
        parse("0:1:explode")
    assert maybe_inject(0, 3, "0:3:nan") is True
    assert maybe_inject(1, 3, "0:3:nan") is False


def _desync(rank, world):
    from hyperion.parallel.debug import assert_replicas_in_sync, assert_same_collective_sequence

    torch.manual_seed(0)
    m = torch.nn.Linear(4, 4)
    assert_replicas_in_sync(m)
    assert_same_collective_sequence("step-1")
    if rank == 1:
        with torch.no_grad():
            m.weight[0, 0] += 1.0
    try:
        assert_replicas_in_sync(m)
        desync = False
    except RuntimeError as e:
        desync = "weight" in str(e)
    try:
        assert_same_collective_sequence("save" if rank == 0 else "train")
        mismatch = False
    except RuntimeError:
        mismatch = True
    return desync, mismatch


def test_desync_and_collective_mismatch_detected():
    res = run_world(_desync, 2)
    assert res[0] == (True, True) and res[1] == (True, True)


def test_killed_rank_fails_the_job_within_timeout(tmp_path):
    """HYPERION_FAULT=1:1:exit kills rank 1 at step 1: the launcher must fail, not hang."""
    env = dict(os.environ, HYPERION_FAULT="1:1:exit", PYTHONPATH=REPO)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "-m", "hyperion.cli.run_distributed", "--model",
           "language_ddp", "--epochs", "1", "--max_steps", "4", "--dataset_size", "512", "--base_dir", str(tmp_path),
           "--no_save"]
    t0 = time.time()
    r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert time.time() - t0 < 280
    assert "injected fault" in r.stderr or "exitcode" in r.stderr


def test_kernel_check_proxy_names_the_faulting_op(monkeypatch):
    """HYPERION_KERNEL_CHECK: every native call is followed by a device sync (outside capture) and
    NaN-producing ops are named (the launch-blocking / sanitizer role)."""
    import torch

    from hyperion.ops import _native

    class Fake:
        __file__ = "fake.so"

        @staticmethod
        def good(x):
            return x * 2

        @staticmethod
        def bad(x):
            return (x * float("nan"), x)

    syncs = []
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: syncs.append(1))
    m = _native.CheckedModule(Fake(), nan=True)
    assert torch.equal(m.good(torch.ones(3)), torch.full((3,), 2.0))
    assert len(syncs) == 1 and m.__file__ == "fake.so"
    try:
        m.bad(torch.ones(3))
    except _native.KernelCheckError as e:
        assert "bad" in str(e) and "NaN" in str(e)
    else:
        raise AssertionError("NaN output not reported")

    def boom(*a):
        raise RuntimeError("HIP error: an illegal memory access was encountered")

    monkeypatch.setattr(torch.cuda, "synchronize", boom)
    try:
        _native.CheckedModule(Fake()).good(torch.ones(1))
    except _native.KernelCheckError as e:
        assert "good" in str(e) and "illegal memory access" in str(e)
    else:
        raise AssertionError("device fault not attributed")
