"""Helpers for multi-process CPU tests (gloo, 127.0.0.1 rendezvous)."""
import io
import os
import socket
import sys
import tempfile
import traceback

import torch
import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, q, store_file=None):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        if store_file is not None:  # file rendezvous: no TCP port to race for under pytest-xdist
            dist.init_process_group("gloo", init_method=f"file://{store_file}", rank=rank, world_size=world)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        out = fn(rank, world, *args)
        buf = io.BytesIO()
        torch.save(out, buf)  # plain bytes: tensors in a Queue would ride on fds that die with the child
        q.put((rank, "ok", buf.getvalue()))
    except BaseException:  # noqa: BLE001
        q.put((rank, "err", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_world(fn, world: int = 2, args=(), timeout: float = 180.0):
    """Run ``fn(rank, world, *args)`` on ``world`` gloo ranks; returns {rank: result}."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    fd, store_file = tempfile.mkstemp(prefix="hyp_dist_", suffix=".store")
    os.close(fd)
    os.unlink(store_file)  # the FileStore creates it; a stale file would hold old keys
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q, store_file)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            rank, status, out = q.get(timeout=timeout)
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{out}")
            res[rank] = torch.load(io.BytesIO(out), weights_only=False)  # our own children's output
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
        if os.path.exists(store_file):
            os.unlink(store_file)
    return res
