"""Checkpoint save / resume (the reference could only save).

Layout keeps the reference's ``{"model_state_dict": ...}`` (``distributed_utils.py:196-199,
274-277,385``) with its key names, and adds what resume needs: ``optimizer_state_dict``,
``scaler_state_dict`` (the real scaler — the reference saved a freshly constructed one,
``mixed_precision.ipynb:278-279``), ``epoch``, ``step``, ``world_size``.

FSDP: ``save_checkpoint`` is COLLECTIVE — every rank enters it.  ``full`` mode all-gathers the
fp32 shards on all ranks and rank 0 writes ``{run_id}_model.pt`` (the reference entered the
gather on rank 0 only: K13); ``sharded`` mode writes ``{run_id}_model_sharded_rank{r}.pt`` per rank
with no communication.  Loading uses ``torch.load(weights_only=True)`` only.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import torch
import torch.distributed as dist
import torch.nn as nn


def _is_fsdp(m: nn.Module) -> bool:
    from ..parallel.fsdp import FullyShardedDataParallel

    return isinstance(m, FullyShardedDataParallel)


def _inner(m: nn.Module) -> nn.Module:
    return getattr(m, "module", m)


def _rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def _save_atomic(doc, path: str) -> None:
    """Write to a temporary name and rename: a crash mid-save never leaves a truncated latest file."""
    tmp = f"{path}.tmp{os.getpid()}"
    torch.save(doc, tmp)
    os.replace(tmp, path)


def save_checkpoint(path: str, model: nn.Module, optimizer: Optional[torch.optim.Optimizer] = None, scaler=None,
                    epoch: int = 0, step: int = 0, mode: str = "full", extra: Optional[Dict[str, Any]] = None) -> Optional[str]:
    """Write a checkpoint; returns the path written on this rank (None on non-writing ranks)."""
    rank = _rank()
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    # every rank, before any branch: the FSDP paths write per-rank files (and the full path only
    # after its all-ranks gather), so a missing directory must not fail there
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    meta = {"epoch": epoch, "step": step, "world_size": world}
    if extra:
        meta.update(extra)
    if _is_fsdp(model):
        if mode == "sharded":
            p = path.replace(".pt", f"_sharded_rank{rank}.pt")
            doc = {"model_sharded_state_dict": model.sharded_state_dict(), **meta}
            if optimizer is not None:
                doc["optimizer_state_dict"] = optimizer.state_dict()
            if scaler is not None:
                doc["scaler_state_dict"] = scaler.state_dict()
            _save_atomic(doc, p)
            return p
        sd = model.full_state_dict(rank0_only=True, offload_to_cpu=True)  # collective on all ranks
        # optimizer state of flat shards is per-rank: store alongside the full model per rank
        if optimizer is not None:
            _save_atomic({"optimizer_state_dict": optimizer.state_dict(), **meta},
                         path.replace(".pt", f"_optim_rank{rank}.pt"))
        if rank != 0:
            return None
        doc = {"model_state_dict": sd, **meta}
        if scaler is not None:
            doc["scaler_state_dict"] = scaler.state_dict()
        _save_atomic(doc, path)
        return path
    if rank != 0:
        return None
    doc = {"model_state_dict": {k: v.detach().cpu() for k, v in _inner(model).state_dict().items()}, **meta}
    if optimizer is not None:
        doc["optimizer_state_dict"] = optimizer.state_dict()
    if scaler is not None:
        doc["scaler_state_dict"] = scaler.state_dict()
    _save_atomic(doc, path)
    return path


def rng_state() -> Dict[str, torch.Tensor]:
    """CPU (+ current GPU) generator states, for bit-exact resume of dropout streams."""
    st = {"rng_cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["rng_cuda"] = torch.cuda.get_rng_state()
    return st


def restore_rng(meta: Dict[str, Any]) -> None:
    if isinstance(meta.get("rng_cpu"), torch.Tensor):
        torch.set_rng_state(meta["rng_cpu"])
    if isinstance(meta.get("rng_cuda"), torch.Tensor) and torch.cuda.is_available():
        torch.cuda.set_rng_state(meta["rng_cuda"])


def load_checkpoint(path: str, model: nn.Module, optimizer: Optional[torch.optim.Optimizer] = None, scaler=None,
                    map_location="cpu") -> Dict[str, Any]:
    """Restore model / optimizer / scaler; returns the metadata (epoch, step, ...)."""
    rank = _rank()
    if _is_fsdp(model):
        sharded = path.replace(".pt", f"_sharded_rank{rank}.pt")
        if os.path.exists(sharded):
            doc = torch.load(sharded, map_location=map_location, weights_only=True)
            model.load_sharded_state_dict(doc["model_sharded_state_dict"])
        else:
            doc = torch.load(path, map_location=map_location, weights_only=True)
            model.load_full_state_dict(doc["model_state_dict"])
            op = path.replace(".pt", f"_optim_rank{rank}.pt")
            if optimizer is not None and os.path.exists(op):
                optimizer.load_state_dict(torch.load(op, map_location=map_location, weights_only=True)["optimizer_state_dict"])
                optimizer = None
    else:
        doc = torch.load(path, map_location=map_location, weights_only=True)
        _inner(model).load_state_dict(doc["model_state_dict"])
    if optimizer is not None and "optimizer_state_dict" in doc:
        optimizer.load_state_dict(doc["optimizer_state_dict"])
    if scaler is not None and "scaler_state_dict" in doc:
        scaler.load_state_dict(doc["scaler_state_dict"])
    return {k: v for k, v in doc.items() if not k.endswith("state_dict")}
