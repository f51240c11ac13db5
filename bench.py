#!/usr/bin/env python3
"""Hyperion-MI355X headline benchmark: ResNet-50 bf16 training throughput (samples/s) and step time.

BASELINE.json metric: "samples/sec + step-ms, ResNet-50 bf16 at 1/2/4/8 MI355X; fused-kernel
speedup".  Config (weak scaling): batch 32 per GPU, 3x224x224 synthetic images, random-init
ResNet-50, bf16 autocast (fp32 master weights), the reference step benchmark's loss/optimizer
(``nn.MSELoss`` vs random (32,1000) targets, ``Adam(lr=1e-3)``: ``Phase 1/baseline_performance.ipynb:
252-358``), data-parallel over RCCL for N>1.  Every timed step does the full forward, backward,
gradient all-reduce (N>1) and optimizer update.

Reference number: 568.22 samples/s = 56.32 ms/step (ResNet-50, batch 32, fp32, 1x MI250X GCD;
``Phase 1/results/benchmarks/Baseline/model_benchmarks.csv:2``).

Usage: ``python bench.py [--gpus N] [--steps K] [--warmup W]``.  For N>1 either run it under
``torch.distributed.run --nproc-per-node N`` (one rank per GPU), or give ``--gpus N`` alone: with
no ``WORLD_SIZE`` in the environment it starts that launcher itself as a CHILD process (before
anything touches the GPU; never an exec) and exits with its return code — rank 0's JSON line
reaches stdout through the inherited file descriptor.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

BASELINE_SAMPLES_PER_S = 568.22  # BASELINE.md §2, ResNet-50 batch 32, 1x MI250X GCD


def parse(argv=None):
    ap = argparse.ArgumentParser(description="Hyperion ResNet-50 training benchmark")
    ap.add_argument("--gpus", type=int, default=None, help="number of GPUs (= WORLD_SIZE)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32, help="per-GPU batch")
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "resnet18"])
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--amp", default="copies", choices=["copies", "autocast"],
                    help="copies = bf16 weight copies + fp32 masters in the fused optimizer; autocast = torch autocast")
    ap.add_argument("--kernels", default=None, choices=["hyperion", "torch"],
                    help="hyperion = fused gfx950 kernels (default); torch = PyTorch eager ops (A/B)")
    ap.add_argument("--graph", type=int, default=1, help="capture the step in a hipGraph (1-GPU; N>1 see --graph-multi)")
    ap.add_argument("--graph-multi", type=int, default=1,
                    help="N>1: capture fwd+bwd and the optimizer as two hipGraphs around eager bucket all-reduces")
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="DDP bucket MiB (default: the all-reduce saturation point of configs/busbw_w{N}.json "
                         "from `test_rccl --sweep --save-tuning`, else 64)")
    ap.add_argument("--ddp-schedule", default="segmented", choices=["segmented", "graph", "split3"],
                    help="N>1 (or --ddp-world1) graphed DDP schedule: segmented (default) = the whole step "
                         "captured as graph segments with each bucket's all-reduce issue / wait as eager holes, "
                         "so every bucket overlaps the rest of the backward; split3 = A/B only, 3 graphs split at "
                         "the model's graph_stages; graph = ONE graph with the RCCL all-reduces recorded into it.  "
                         "Measured at world 1 with the native RCCL communicator: "
                         "5.15 vs 14.5 ms/step (profiles/r05/ddp_schedule_ab.json)")
    ap.add_argument("--ddp-world1", type=int, default=0,
                    help="A/B only: wrap the 1-GPU model in DDP with buckets and the native RCCL communicator "
                         "(the N>1 schedule's collectives at world 1)")
    ap.add_argument("--comm-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--channels-last", type=int, default=1)
    ap.add_argument("--loss", default="head", choices=["torch", "fused", "head"],
                    help="MSE loss: torch's ops, Hyperion's one-pass kernel, or 'head': the classifier fc and "
                         "the MSE as one fused native forward + one backward launch (ops.losses.LinearMSELoss)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--smi", type=int, default=0, help="sample amd-smi power / clocks during the timed steps")
    return ap.parse_args(argv)


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args, argv) -> "int | None":
    """``--gpus N`` (N > 1) outside a launcher: one rank per GPU via torch.distributed.run, as a
    child process.  Returns its exit code, or None when this process is already a rank."""
    if args.gpus is None or args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL between the ranks
    return subprocess.call(cmd, env=env)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    rc = self_launch(args, argv)
    if rc is not None:
        return rc
    if args.kernels:
        os.environ["HYPERION_KERNELS"] = args.kernels
    import torch
    import torch.distributed as dist
    import torch.nn as nn

    import hyperion
    from hyperion.models import resnet18, resnet50
    from hyperion.ops import FusedAdam, _native
    from hyperion.parallel import DDP, init_from_env
    from hyperion.train.step import TrainStep
    from hyperion.utils import seed_everything

    # HYPERION_DIST_BACKEND=gloo (+ HYPERION_COMM=torch): rehearse the N>1 path with several ranks on one GPU
    env = init_from_env(backend=os.environ.get("HYPERION_DIST_BACKEND") or None)
    n_gpus = env.world_size
    if args.gpus is not None and args.gpus != n_gpus and env.rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={n_gpus}; using WORLD_SIZE", file=sys.stderr)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    seed_everything(1234, env.rank)
    torch.backends.cudnn.benchmark = True

    amp = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": None}[args.precision]
    model = (resnet50 if args.model == "resnet50" else resnet18)(num_classes=1000).to(dev)
    mf = torch.channels_last if args.channels_last else torch.contiguous_format
    model = model.to(memory_format=mf)
    copies = amp is not None and args.amp == "copies"
    if copies:
        from hyperion.train.amp import cast_for_compute

        cast_for_compute(model, amp)
    if n_gpus > 1 or args.ddp_world1:
        # fp32 gradient buckets by default (the reference reduced fp32 grads); --comm-dtype bf16 opt-in
        kw = {}
        if n_gpus == 1:
            from hyperion.bench.models import _ensure_pg
            from hyperion.parallel.comm import NativeComm

            _ensure_pg()  # a world-1 process group for the communicator's bootstrap
            # HYPERION_COMM=torch: torch.distributed's world-1 no-op all-reduce (isolates the
            # segment-boundary cost from the native RCCL issue / wait)
            comm = None if os.environ.get("HYPERION_COMM") == "torch" else NativeComm(dev)
            kw = dict(buckets_at_world_1=True, comm=comm)
        model = DDP(model, bucket_cap_mb=args.bucket_mb, broadcast_buffers=False,
                    comm_dtype=torch.bfloat16 if args.comm_dtype == "bf16" else torch.float32, **kw)
    opt = FusedAdam(model.parameters(), lr=1e-3, zero_grad_in_step=True)
    # the reference's nn.MSELoss (mean) — Hyperion's fused forward+gradient pass on gfx950
    from hyperion.ops.losses import MSELoss

    loss_fn = MSELoss() if (args.kernels != "torch" and args.loss == "fused") else nn.MSELoss()
    if args.kernels != "torch" and args.loss == "head" and dev.type == "cuda":
        from hyperion.ops.losses import LinearMSELoss

        net = model.module if hasattr(model, "module") else model
        net.head_in_loss = True  # the model returns pooled features; the loss applies fc (same math)
        loss_fn = LinearMSELoss(net.fc)

    B = args.batch
    x = torch.rand(B, 3, args.image, args.image, device=dev).to(memory_format=mf)
    if copies:
        x = x.to(amp)
    y = torch.rand(B, 1000, device=dev)
    use_graph = bool(args.graph) and dev.type == "cuda" and (n_gpus == 1 or bool(args.graph_multi))
    step = TrainStep(model, opt, loss_fn, amp_dtype=None if copies else amp, graph=use_graph,
                     ddp_schedule=args.ddp_schedule)

    for _ in range(args.warmup):
        step(x, y)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    if n_gpus > 1:
        dist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    smi = None
    if args.smi and env.rank == 0:
        from hyperion.profiling.smi import SmiSampler

        smi = SmiSampler(interval_s=0.5).__enter__()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step(x, y)
    host_s = time.perf_counter() - t0  # launch-side time of the timed loop (before the final sync)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    if n_gpus > 1:
        dist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if smi is not None:
        smi.__exit__(None, None, None)
    if n_gpus > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.float().item())
    replicas = None
    if n_gpus > 1:
        # correctness self-check after the timed loop: every rank must hold bit-identical weights
        from hyperion.parallel.debug import assert_replicas_in_sync

        try:
            replicas = {"in_sync": True, "tensors": assert_replicas_in_sync(model)}
        except RuntimeError as e:
            replicas = {"in_sync": False, "error": str(e)[:300]}
    ms = elapsed / args.steps * 1e3
    value = n_gpus * B * args.steps / elapsed
    if env.rank == 0:
        rec = {
            "metric": "resnet50_train_samples_per_sec" if args.model == "resnet50" else "resnet18_train_samples_per_sec",
            "value": round(value, 2),
            "unit": "samples/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_SAMPLES_PER_S, 3) if args.model == "resnet50" else None,
            "dtype": args.precision,
            "data": f"synthetic (torch.rand images 3x{args.image}x{args.image}, rand targets; random-init weights)",
            "config": {
                "model": args.model,
                "global_batch": B * n_gpus,
                "per_gpu_batch": B,
                "seq_len": None,
                "image": args.image,
                "parallelism": f"dp{n_gpus}",
                "loss": "MSE vs rand(B,1000) (reference benchmark_model)" + (
                    "; fc + MSE fused (linear_mse.hip)" if args.loss == "head" else ""),
                "optimizer": "Adam lr=1e-3 (hyperion FusedAdam, multi-tensor)",
                "hipgraph": use_graph,
                "ddp_schedule": (None if (n_gpus == 1 and not args.ddp_world1) else
                                 f"segmented: {step.seg.num_segments} graph segments, bucket all-reduce holes"
                                 if step.seg is not None else
                                 "one graph, bucket all-reduces captured on the comm stream"
                                 if args.ddp_schedule == "graph" and use_graph else
                                 "3 graphs: top fwd+bwd | bottom bwd overlapping the top buckets' RCCL all-reduce | optimizer"
                                 if step.graph3 is not None else
                                 "2 graphs around eager bucket all-reduces" if step.graph2 is not None else
                                 "eager, all-reduce overlapped with backward"),
                "amp": ("bf16 compute copies + fp32 master weights" if copies else
                        ("torch.autocast " + args.precision if amp is not None else "none")),
                "kernels": _native.backend(),
                "native_so": _native.loaded_path(),
                "channels_last": bool(args.channels_last),
                "grad_allreduce_dtype": (args.comm_dtype if (n_gpus > 1 or args.ddp_world1) else None),
                "bucket_mb": getattr(model, "bucket_cap_mb", None),
            },
            "baseline": {"value": BASELINE_SAMPLES_PER_S, "ms_per_step": 56.32, "hw": "1x MI250X GCD, fp32"},
            "final_loss": round(final_loss, 6),
            # host time per step issuing the timed loop: close to ms_per_step means launch-bound
            "host_ms_per_step": round(host_s / args.steps * 1e3, 3),
        }
        if replicas is not None:
            rec["replicas"] = replicas
        if smi is not None:
            rec["smi"] = smi.summary()
        if os.environ.get("HYPERION_SEG_PROFILE") == "1" and getattr(step, "seg", None) is not None:
            rec["seg_host_profile"] = step.seg.host_profile()
        line = json.dumps(rec)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if n_gpus > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
