"""Single-GPU trainers and probes with the notebooks' APIs.

Reference functions and where they live:
* ``train_language_model(model, dataloader, device, epochs)`` / ``train_cifar_model`` —
  fp32, AdamW (2e-4 / 1e-3), CE(ignore pad) — ``core_framework.ipynb:243-284``;
* ``train_language_model_amp`` / ``train_cifar_model_amp`` — fp16 autocast + GradScaler —
  ``mixed_precision.ipynb:121-171``;
* ``profile_amp_training(model, dataloader, device, n_batches=10)`` — wall time + peak memory —
  ``mixed_precision.ipynb:314-341`` (the reference called ``model.eval()`` while "training";
  here the model stays in train mode);
* ``print_memory`` / ``train_one_batch`` — ``memory_optimization.ipynb:152-176,345-379`` (the
  reference reported memory allocated after the step, not peak; both are returned here).

Differences: no per-step ``loss.item()`` host sync (losses accumulate on device), the LM path uses
the fused head+CE when the model provides ``forward_loss``, AMP state (the real scaler) is
returned for checkpointing.
"""
from __future__ import annotations

import time
from typing import Dict, List

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..models.simple_lm import GPT2_PAD
from ..ops.optim import FusedAdam
from .amp import LossScaler


def _lm_loss(model: nn.Module, ids: torch.Tensor, pad: int) -> torch.Tensor:
    x, y = ids[:, :-1], ids[:, 1:]
    if hasattr(model, "forward_loss"):
        return model.forward_loss(x, y, ignore_index=pad)
    logits = model(x)
    return F.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), y.reshape(-1), ignore_index=pad)


def _run(model, dataloader, device, epochs, lr, kind, amp_dtype=None, pad=GPT2_PAD, max_steps=None,
         log=print) -> Dict:
    model.to(device).train()
    opt = FusedAdam(model.parameters(), lr=lr, weight_decay=0.01, adamw=True)
    use_scaler = amp_dtype == torch.float16 and device.type == "cuda"
    scaler = LossScaler(enabled=use_scaler, device=device)
    history: List[Dict] = []
    for ep in range(epochs):
        t0 = time.time()
        tot = torch.zeros((), device=device)
        correct = torch.zeros((), device=device)
        seen = torch.zeros((), device=device)
        n = 0
        for i, batch in enumerate(dataloader):
            if max_steps is not None and i >= max_steps:
                break
            opt.zero_grad(set_to_none=True)
            with torch.autocast(device.type, dtype=amp_dtype or torch.float32,
                                enabled=amp_dtype is not None and not (device.type == "cpu" and amp_dtype == torch.float16)):
                if kind == "lm":
                    ids = batch[0].to(device, non_blocking=True)
                    loss = _lm_loss(model, ids, pad)
                else:
                    img, lbl = batch[0].to(device, non_blocking=True), batch[1].to(device, non_blocking=True)
                    logits = model(img)
                    loss = F.cross_entropy(logits.float(), lbl)
                    correct += (logits.argmax(1) == lbl).sum()
                    seen += lbl.numel()
            if use_scaler:
                scaler.scale(loss).backward()
                scaler.step(opt)
                scaler.update()
            else:
                loss.backward()
                opt.step()
            tot += loss.detach().float()
            n += 1
        rec = {"epoch": ep + 1, "loss": (tot / max(n, 1)).item(), "time_s": time.time() - t0, "steps": n}
        if kind == "cifar":
            rec["accuracy"] = (correct / seen.clamp_min(1)).item() * 100
        history.append(rec)
        log(f"epoch {ep + 1}: " + ", ".join(f"{k}={v:.4f}" if isinstance(v, float) else f"{k}={v}" for k, v in rec.items()))
    return {"history": history, "optimizer": opt, "scaler": scaler}


def train_language_model(model, dataloader, device, epochs: int = 1, **kw) -> Dict:
    return _run(model, dataloader, torch.device(device), epochs, 2e-4, "lm", None, **kw)


def train_cifar_model(model, dataloader, device, epochs: int = 1, **kw) -> Dict:
    return _run(model, dataloader, torch.device(device), epochs, 1e-3, "cifar", None, **kw)


def train_language_model_amp(model, dataloader, device, epochs: int = 3, dtype=torch.float16, **kw) -> Dict:
    return _run(model, dataloader, torch.device(device), epochs, 2e-4, "lm", dtype, **kw)


def train_cifar_model_amp(model, dataloader, device, epochs: int = 3, dtype=torch.float16, **kw) -> Dict:
    return _run(model, dataloader, torch.device(device), epochs, 1e-3, "cifar", dtype, **kw)


def profile_amp_training(model, dataloader, device, n_batches: int = 10, dtype=torch.float16) -> Dict:
    """Wall time and peak memory of ``n_batches`` AMP training steps (model stays in train mode)."""
    device = torch.device(device)
    if device.type == "cuda":
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(device)
    t0 = time.time()
    _run(model, dataloader, device, 1, 2e-4, "lm", dtype, max_steps=n_batches, log=lambda s: None)
    if device.type == "cuda":
        torch.cuda.synchronize()
    return {"time_s": time.time() - t0,
            "peak_mem_mb": torch.cuda.max_memory_allocated(device) / 2**20 if device.type == "cuda" else 0.0}


def print_memory(prefix: str = "") -> Dict[str, float]:
    from ..utils.device import get_gpu_memory

    m = get_gpu_memory()
    print(f"{prefix} allocated {m['allocated_mb']:.2f} MB | reserved {m['reserved_mb']:.2f} MB | peak {m['peak_mb']:.2f} MB")
    return m


def train_one_batch(model, dataloader, device, kind: str = "lm") -> Dict[str, float]:
    """One training step; returns allocated-after (reference metric) AND true peak memory."""
    device = torch.device(device)
    model.to(device).train()
    if device.type == "cuda":
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(device)
    _run(model, dataloader, device, 1, 1e-3, kind, None, max_steps=1, log=lambda s: None)
    if device.type != "cuda":
        return {"allocated_after_mb": 0.0, "peak_mb": 0.0}
    torch.cuda.synchronize()
    return {"allocated_after_mb": torch.cuda.memory_allocated(device) / 2**20,
            "peak_mb": torch.cuda.max_memory_allocated(device) / 2**20}


