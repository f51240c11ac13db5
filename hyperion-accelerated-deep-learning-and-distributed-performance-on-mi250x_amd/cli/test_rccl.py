"""RCCL sanity check + bus-bandwidth sweep (replaces the reference's ``test_nccl.py``).

The reference all-reduced ``ones(1) * local_rank`` once with a 30 s timeout and printed the result
without checking it (``02_development/test_nccl.py:8-47``).  This version ASSERTS the sum
(w(w-1)/2) and the other collectives' results, then (``--sweep``) measures algorithm / bus
bandwidth of all_reduce, all_gather, reduce_scatter over message sizes with hipEvents — the curve
DDP bucket and FSDP unit sizes are chosen from (7 xGMI links × ≈153 GB/s per GPU).

``--backend native`` (default on GPU) runs the checks and the sweep through Hyperion's own C++ RCCL
communicator (``parallel/comm.py`` ``NativeComm`` — the one DDP / FSDP use), ``--backend torch``
through ``torch.distributed`` (ProcessGroupNCCL on GPU, gloo on CPU).

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


def _comm(backend: str, device: torch.device):
    from hyperion.parallel.comm import NativeComm, TorchComm

    return NativeComm(device) if backend == "native" else TorchComm()


def _run(work) -> None:
    if work is not None:
        work.wait()


def check(rank: int, world: int, device: torch.device, comm=None) -> None:
    from hyperion.parallel.comm import TorchComm

    comm = comm or TorchComm()
    t = torch.ones(1, device=device) * rank
    _run(comm.all_reduce(t, "sum"))
    want = world * (world - 1) / 2
    assert float(t.item()) == want, f"all_reduce: got {t.item()} want {want}"
    big = torch.full((1 << 20,), float(rank + 1), device=device, dtype=torch.float32)
    _run(comm.all_reduce(big, "avg"))
    assert big.eq((world + 1) / 2).all(), f"all_reduce avg: {big[:4].tolist()}"
    g = torch.empty(world, device=device)
    _run(comm.all_gather(g, torch.full((1,), float(rank), device=device)))
    assert g.tolist() == [float(i) for i in range(world)], f"all_gather: {g.tolist()}"
    rs = torch.empty(1, device=device)
    _run(comm.reduce_scatter(rs, torch.arange(world, dtype=torch.float32, device=device), "sum"))
    assert float(rs.item()) == rank * world, f"reduce_scatter: {rs.item()}"
    b = torch.full((4,), float(rank), device=device)
    _run(comm.broadcast(b, 0))
    assert b.eq(0).all(), "broadcast"
    a2a_in = torch.arange(world, dtype=torch.float32, device=device) + 100 * rank
    a2a = torch.empty(world, device=device)
    _run(comm.all_to_all(a2a, a2a_in))
    assert a2a.tolist() == [float(100 * j + rank) for j in range(world)], f"all_to_all: {a2a.tolist()}"
    if rank == 0:
        print(f"[test_rccl] world={world} backend={getattr(comm, 'backend', '?')}: all_reduce (sum, avg) / all_gather"
              " / reduce_scatter / broadcast / all_to_all OK", flush=True)


def sweep(rank: int, world: int, device: torch.device, sizes_mb, iters: int = 20, dtype=torch.bfloat16, comm=None):
    """busbw per NCCL-tests conventions: AR 2(n-1)/n, AG/RS (n-1)/n of algbw."""
    from hyperion.parallel.comm import TorchComm

    comm = comm or TorchComm()
    rows = []
    es = torch.empty((), dtype=dtype).element_size()
    for mb in sizes_mb:
        n = max(world, int(mb * 2**20 / es) // world * world)
        x = torch.ones(n, dtype=dtype, device=device)
        shard = torch.empty(n // world, dtype=dtype, device=device)
        for name, fn, factor in (
            ("all_reduce", lambda: _run(comm.all_reduce(x, "sum")), 2 * (world - 1) / world),
            ("all_gather", lambda: _run(comm.all_gather(x, shard)), (world - 1) / world),
            ("reduce_scatter", lambda: _run(comm.reduce_scatter(shard, x, "sum")), (world - 1) / world),
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
            rows.append({"op": name, "backend": getattr(comm, "backend", "?"), "bytes": n * es, "time_us": t * 1e6,
                         "algbw_GBps": algbw, "busbw_GBps": algbw * factor})
            if rank == 0:
                print(f"{name:15s} {n * es / 2**20:10.1f} MiB  {t * 1e6:10.1f} us  algbw {algbw:8.1f}  busbw {algbw * factor:8.1f} GB/s")
    return rows


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--sizes_mb", default="0.25,1,4,16,64,256,1024")
    ap.add_argument("--timeout", type=float, default=60.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--save-tuning", action="store_true",
                    help="also write configs/busbw_w{world}.json: DDP then sizes its buckets from this curve "
                         "(parallel/tuning.py)")
    ap.add_argument("--backend", default=None, choices=["torch", "native"],
                    help="collectives through Hyperion's C++ RCCL communicator (native, GPU default) or torch.distributed")
    a = ap.parse_args(argv)
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    gpu = torch.cuda.is_available()
    # HYPERION_SAME_DEVICE=1: every rank on GPU 0 (rehearsing several ranks on a one-GPU box)
    dev_index = 0 if os.environ.get("HYPERION_SAME_DEVICE") == "1" else local
    device = torch.device("cuda", dev_index) if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(device)
    try:
        dist.init_process_group("nccl" if gpu else "gloo", timeout=datetime.timedelta(seconds=a.timeout),
                                **({"device_id": device} if gpu else {}))
        backend = a.backend or ("native" if gpu else "torch")
        if backend == "native" and not gpu:
            raise RuntimeError("--backend native needs GPUs (RCCL)")
        comm = _comm(backend, device)
        check(rank, world, device, comm)
        if a.sweep and gpu:
            rows = sweep(rank, world, device, [float(s) for s in a.sizes_mb.split(",")], comm=comm)
            outs = [a.out] if a.out else []
            if a.save_tuning:
                from hyperion.parallel.tuning import sweep_path

                outs.append(sweep_path(world))
            for path in outs if rank == 0 else []:
                with open(path, "w") as f:
                    json.dump({"world": world, "rows": rows}, f, indent=2)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        print(f"[test_rccl] rank {rank} FAILED: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
