"""RCCL sanity check + bus-bandwidth sweep (replaces the reference's ``test_nccl.py``).

The reference all-reduced ``ones(1) * local_rank`` once with a 30 s timeout and printed the result
without checking it (``02_development/test_nccl.py:8-47``).  This version ASSERTS the sum
(w(w-1)/2) and the other collectives' results, then (``--sweep``) measures algorithm / bus
bandwidth of all_reduce, all_gather, reduce_scatter over message sizes with hipEvents — the curve
DDP bucket and FSDP unit sizes are chosen from (7 xGMI links × ≈153 GB/s per GPU).

    torchrun --standalone --nproc-per-node 8 -m hyperion.cli.test_rccl [--sweep] [--backend torch|native]
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys

import torch
import torch.distributed as dist


def check(rank: int, world: int, device: torch.device) -> None:
    t = torch.ones(1, device=device) * rank
    dist.all_reduce(t)
    want = world * (world - 1) / 2
    assert float(t.item()) == want, f"all_reduce: got {t.item()} want {want}"
    g = torch.empty(world, device=device)
    dist.all_gather_into_tensor(g, torch.full((1,), float(rank), device=device))
    assert g.tolist() == [float(i) for i in range(world)], f"all_gather: {g.tolist()}"
    rs = torch.empty(1, device=device)
    dist.reduce_scatter_tensor(rs, torch.arange(world, dtype=torch.float32, device=device))
    assert float(rs.item()) == rank * world, f"reduce_scatter: {rs.item()}"
    b = torch.full((4,), float(rank), device=device)
    dist.broadcast(b, src=0)
    assert b.eq(0).all(), "broadcast"
    if rank == 0:
        print(f"[test_rccl] world={world}: all_reduce / all_gather / reduce_scatter / broadcast OK")


def sweep(rank: int, world: int, device: torch.device, sizes_mb, iters: int = 20, dtype=torch.bfloat16):
    """busbw per NCCL-tests conventions: AR 2(n-1)/n, AG/RS (n-1)/n of algbw."""
    rows = []
    es = torch.empty((), dtype=dtype).element_size()
    for mb in sizes_mb:
        n = max(world, int(mb * 2**20 / es) // world * world)
        x = torch.ones(n, dtype=dtype, device=device)
        shard = torch.empty(n // world, dtype=dtype, device=device)
        for name, fn, factor in (
            ("all_reduce", lambda: dist.all_reduce(x), 2 * (world - 1) / world),
            ("all_gather", lambda: dist.all_gather_into_tensor(x, shard), (world - 1) / world),
            ("reduce_scatter", lambda: dist.reduce_scatter_tensor(shard, x), (world - 1) / world),
        ):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                fn()
            e.record()
            e.synchronize()
            t = s.elapsed_time(e) / iters / 1e3
            t_max = torch.tensor([t], device=device)
            dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
            t = float(t_max.item())
            algbw = n * es / t / 1e9
            rows.append({"op": name, "bytes": n * es, "time_us": t * 1e6, "algbw_GBps": algbw,
                         "busbw_GBps": algbw * factor})
            if rank == 0:
                print(f"{name:15s} {n * es / 2**20:10.1f} MiB  {t * 1e6:10.1f} us  algbw {algbw:8.1f}  busbw {algbw * factor:8.1f} GB/s")
    return rows


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--sizes_mb", default="0.25,1,4,16,64,256,1024")
    ap.add_argument("--timeout", type=float, default=60.0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    gpu = torch.cuda.is_available()
    device = torch.device("cuda", local) if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(device)
    try:
        dist.init_process_group("nccl" if gpu else "gloo", timeout=datetime.timedelta(seconds=a.timeout),
                                **({"device_id": device} if gpu else {}))
        check(rank, world, device)
        if a.sweep and gpu:
            rows = sweep(rank, world, device, [float(s) for s in a.sizes_mb.split(",")])
            if rank == 0 and a.out:
                with open(a.out, "w") as f:
                    json.dump({"world": world, "rows": rows}, f, indent=2)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        print(f"[test_rccl] rank {rank} FAILED: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
