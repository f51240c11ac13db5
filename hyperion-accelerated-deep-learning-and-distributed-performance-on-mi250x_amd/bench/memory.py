"""Memory probes: activation checkpointing and AMP memory.

Reference (``memory_optimization.ipynb:152-176, 303-319, 345-379``; ``mixed_precision.ipynb:314-341``):
no-grad forward memory of the LM and ResNet before/after checkpointing (under ``no_grad``, so
checkpointing could not matter — warning at :290), and one-batch training memory measured as
``memory_allocated`` AFTER the step (478.68 MB → 587.06 MB "with" checkpointing), not peak.

``checkpoint_memory_probe`` reports both numbers for both settings: the reference metric
(allocated after the step) and the meaningful one (peak during forward+backward, which is what
checkpointing lowers), plus step time so the recompute cost is visible.
"""
from __future__ import annotations

import time
from typing import Callable, Dict

import torch
import torch.nn as nn


def _measure(step: Callable[[], None], dev: torch.device) -> Dict[str, float]:
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    base = torch.cuda.memory_allocated(dev)
    torch.cuda.reset_peak_memory_stats(dev)
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize(dev)
    return {"time_ms": (time.perf_counter() - t0) * 1e3,
            "peak_mb": (torch.cuda.max_memory_allocated(dev) - base) / 2**20,
            "allocated_after_mb": torch.cuda.memory_allocated(dev) / 2**20}


def checkpoint_memory_probe(kind: str = "lm", batch: int = 32, precision: str = "bf16") -> Dict[str, Dict]:
    from ..models.resnet import resnet18
    from ..models.simple_lm import GPT2_PAD, simple_lm_256
    from ..train.checkpointing import checkpoint_resnet_blocks

    dev = torch.device("cuda")
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": None}[precision]
    out = {}
    for ckpt in (False, True):
        torch.manual_seed(0)
        if kind == "lm":
            m = simple_lm_256(use_checkpoint=ckpt).to(dev)
            ids = torch.randint(0, 50257, (batch, 128), device=dev)

            def step():
                with torch.autocast("cuda", dtype=dt or torch.float32, enabled=dt is not None):
                    loss = m.forward_loss(ids[:, :-1], ids[:, 1:], ignore_index=GPT2_PAD)
                loss.backward()
        else:
            m = resnet18(num_classes=10).to(dev).to(memory_format=torch.channels_last)
            if ckpt:
                checkpoint_resnet_blocks(m)
            x = torch.randn(batch, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)
            y = torch.randint(0, 10, (batch,), device=dev)

            def step():
                with torch.autocast("cuda", dtype=dt or torch.float32, enabled=dt is not None):
                    loss = nn.functional.cross_entropy(m(x).float(), y)
                loss.backward()
        step()  # warm-up (allocator, kernel selection)
        m.zero_grad(set_to_none=True)
        out["checkpointed" if ckpt else "baseline"] = _measure(step, dev)
        del m
    return out
