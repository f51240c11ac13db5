"""Launcher CLI, flag-compatible with the reference's ``run_distributed.py``.

    torchrun --standalone --nproc-per-node N -m hyperion.cli.run_distributed \
        --model {language_ddp,cifar,language_fsdp,gpt2_fsdp,llama,all,scaling} --epochs 5 --base_dir . \
        [--hf_token T] [--model_id ID] [--lora] [--batch_size 1] [--progress_every 50] [--scaling_gpus 1,2,4,8]

Reference behaviour (``run_distributed.py:38-149``): reads RANK/WORLD_SIZE/LOCAL_RANK from the env,
dispatches one trainer, ``all`` runs the four trainers in sequence, ``scaling`` makes rank 0 start
NESTED torchrun jobs while the outer group is alive, and rank 0 always ends with
``create_scaling_report``.  Here ``scaling`` runs only when launched as a single process (it is
the top-level orchestrator, ``bench.scaling.run_scaling_experiment``) and refuses to nest.
Extra flags: ``--synthetic/--real-data``, ``--precision``, ``--kernels {hyperion,torch}``,
``--max_steps``, ``--dataset_size``, ``--resume``, ``--ckpt_mode``, ``--seed``, ``--config FILE``.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
from typing import List, Optional


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Hyperion-MI355X distributed training launcher")
    ap.add_argument("--model", default="language_ddp",
                    choices=["language_ddp", "cifar", "language_fsdp", "gpt2_fsdp", "llama", "all", "scaling"],
                    help="gpt2_fsdp: GPT-2-small causal LM, FSDP with per-layer units (BASELINE config 4)")
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--base_dir", default=os.getcwd())
    ap.add_argument("--hf_token", default=None)
    ap.add_argument("--model_id", default="NousResearch/Llama-2-7b-hf")
    ap.add_argument("--lora", action="store_true")
    ap.add_argument("--batch_size", type=int, default=1, help="Llama per-rank batch (reference default 1)")
    ap.add_argument("--lm_batch_size", type=int, default=None, help="gpt2_fsdp per-rank batch (default 32)")
    ap.add_argument("--progress_every", type=int, default=50)
    ap.add_argument("--scaling_gpus", default="1,2,4,8")
    # hyperion extensions
    ap.add_argument("--config", default=None, help="YAML/JSON config file (hyperion.config)")
    ap.add_argument("--real-data", dest="synthetic", action="store_false",
                    help="read data/processed/* like the reference (default: synthetic of the same shapes)")
    ap.add_argument("--precision", default=None, choices=["fp32", "fp16", "bf16"])
    ap.add_argument("--kernels", default=None, choices=["hyperion", "torch"])
    ap.add_argument("--max_steps", type=int, default=None, help="cap steps per epoch")
    ap.add_argument("--dataset_size", type=int, default=None)
    ap.add_argument("--resume", default=None, help="checkpoint path, or 'auto' = this run kind's latest checkpoint")
    ap.add_argument("--ckpt_every", type=int, default=None, help="write the latest checkpoint every N steps")
    ap.add_argument("--max_restarts", type=int, default=0,
                    help="single process: run each attempt in a FRESH child process and re-run a failed trainer up "
                         "to N times with --resume auto (the supervising parent never touches the GPU); "
                         "multi-process: use torchrun --max-restarts N together with --resume auto")
    ap.add_argument("--ckpt_mode", default="full", choices=["full", "sharded"])
    ap.add_argument("--lora_parallel", default="fsdp", choices=["fsdp", "ddp"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no_save", action="store_true")
    ap.add_argument("--causal", action="store_true", help="causal mask for the LM (reference had none)")
    return ap


def _env():
    try:
        return int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ.get("LOCAL_RANK", 0))
    except KeyError:
        return None


def _child_argv(argv: List[str], model: str, resume: Optional[str]) -> List[str]:
    """``argv`` without --max_restarts, with --model pinned to ``model`` and --resume to ``resume``."""
    out, skip = [], False
    for i, a in enumerate(argv):
        if skip:
            skip = False
            continue
        key = a.split("=", 1)[0]
        if key in ("--max_restarts", "--model", "--resume"):
            skip = "=" not in a
            continue
        out.append(a)
    out += ["--model", model]
    if resume:
        out += ["--resume", resume]
    return out


def _repo_root() -> str:
    """Directory holding the ``hyperion`` import shim (so the child resolves the same package)."""
    import hyperion

    src = getattr(hyperion, "_SRC", None) or os.path.dirname(os.path.abspath(hyperion.__file__))
    return os.path.dirname(src)


def supervise(argv: List[str], models: List[str], max_restarts: int, resume: Optional[str]) -> int:
    """Restart policy for a single-process run: each attempt is a NEW interpreter, so a
    sticky HIP fault, an aborted communicator, captured graphs or module-global caches of the failed
    attempt can never leak into the retry.  This process only waits on children."""
    for m in models:
        attempt, res = 0, resume
        while True:
            cmd = [sys.executable, "-m", "hyperion.cli.run_distributed"] + _child_argv(argv, m, res)
            env = dict(os.environ, HYPERION_RESTART_ATTEMPT=str(attempt))
            env["PYTHONPATH"] = os.pathsep.join(p for p in (_repo_root(), env.get("PYTHONPATH", "")) if p)
            rc = subprocess.run(cmd, env=env).returncode
            if rc == 0:
                break
            if attempt >= max_restarts:
                print(f"[run_distributed] {m} failed (exit {rc}); no restarts left", file=sys.stderr, flush=True)
                return rc
            attempt += 1
            res = "auto"
            print(f"[run_distributed] {m} failed (exit {rc}); restart {attempt}/{max_restarts} in a fresh process "
                  "from the latest checkpoint", file=sys.stderr, flush=True)
    return 0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = build_parser().parse_args(argv)
    if args.config:
        from hyperion.config import apply_to_args, load_config

        apply_to_args(load_config(args.config), args)
    if args.kernels:
        os.environ["HYPERION_KERNELS"] = args.kernels
    if args.hf_token:
        os.environ.setdefault("HF_TOKEN", args.hf_token)  # accepted; nothing is downloaded
    from hyperion.bench.scaling import create_scaling_report, run_scaling_experiment
    from hyperion.train.distributed import RunOptions

    env = _env()
    if args.model == "scaling":
        if env is not None and env[1] > 1:
            print("--model scaling is a top-level orchestrator; run it as a single process (no nested torchrun)")
            return 2
        extra = []
        for flag in ("precision", "kernels", "max_steps", "dataset_size"):
            v = getattr(args, flag)
            if v is not None:
                extra += [f"--{flag}", str(v)]
        for m in ("language_ddp", "cifar", "language_fsdp", "llama"):
            run_scaling_experiment(m, [int(g) for g in args.scaling_gpus.split(",")], args.epochs, args.base_dir,
                                   args.hf_token, extra_args=extra + (["--lora"] if m == "llama" and args.lora else []))
        return 0
    if env is None:
        env = (0, 1, 0)  # plain `python -m`: a single process (the reference exited here)
    rank, world, _local = env
    todo = ["language_ddp", "cifar", "language_fsdp", "llama"] if args.model == "all" else [args.model]
    if args.max_restarts > 0:
        if world > 1:
            print("--max_restarts is for single-process runs; with torchrun use --max-restarts N and --resume auto",
                  file=sys.stderr)
            return 2
        return supervise(argv, todo, args.max_restarts, args.resume)
    opts = RunOptions(synthetic=args.synthetic, dataset_size=args.dataset_size, max_steps_per_epoch=args.max_steps,
                      precision=args.precision, seed=args.seed, save=not args.no_save, ckpt_mode=args.ckpt_mode,
                      resume=args.resume, causal=args.causal, ckpt_every=args.ckpt_every)
    for m in todo:
        _run_one(m, rank, world, args, opts)
    if rank == 0:
        create_scaling_report(os.path.join(args.base_dir, "data", "distributed"))
    return 0


def _run_one(m: str, rank: int, world: int, args, opts) -> None:
    from hyperion.train.distributed import (train_cifar_model_ddp, train_gpt2_fsdp, train_language_model_ddp,
                                            train_language_model_fsdp, train_llama_fsdp)

    if m == "language_ddp":
        train_language_model_ddp(rank, world, args.epochs, args.base_dir, opts)
    elif m == "cifar":
        train_cifar_model_ddp(rank, world, args.epochs, args.base_dir, opts)
    elif m == "language_fsdp":
        train_language_model_fsdp(rank, world, args.epochs, args.base_dir, opts)
    elif m == "gpt2_fsdp":
        train_gpt2_fsdp(rank, world, args.epochs, args.base_dir, opts, batch_size=args.lm_batch_size or 32)
    elif m == "llama":
        train_llama_fsdp(rank, world, epochs=args.epochs, base_dir=args.base_dir, hf_token=args.hf_token,
                         model_id=args.model_id, lora=args.lora, batch_size=args.batch_size,
                         progress_every=args.progress_every, opts=opts, lora_parallel=args.lora_parallel)


if __name__ == "__main__":
    sys.exit(main())
