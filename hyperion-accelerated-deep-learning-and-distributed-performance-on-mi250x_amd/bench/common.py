"""Generic benchmarking helpers — the reference's orphan library, made usable.

Reference: ``Phase 1/benchmarking.py`` (never imported there): ``benchmark_forward_pass``
(:12-55), ``benchmark_training_step`` with optional fp16 AMP + GradScaler (:57-151),
``compare_precision_formats`` (:153-221), ``save_benchmark_results`` (:223-239).  Same
signatures and result keys; timing brackets synchronize as the reference did.
"""
from __future__ import annotations

import os
import time
from typing import Callable, Dict, List, Sequence

import torch
import torch.nn as nn


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def benchmark_forward_pass(model: nn.Module, inputs: torch.Tensor, num_iterations: int = 50, warmup: int = 10) -> Dict:
    model.eval()
    with torch.no_grad():
        for _ in range(warmup):
            model(inputs)
        _sync()
        t0 = time.perf_counter()
        for _ in range(num_iterations):
            model(inputs)
        _sync()
    total = time.perf_counter() - t0
    avg = total / num_iterations
    return {"total_time": total, "avg_time": avg, "throughput": inputs.shape[0] / avg}


def benchmark_training_step(model: nn.Module, inputs: torch.Tensor, targets: torch.Tensor, optimizer,
                            criterion, num_iterations: int = 50, warmup: int = 10, use_amp: bool = False,
                            amp_dtype: torch.dtype = torch.float16) -> Dict:
    from ..train.amp import LossScaler

    model.train()
    dev = inputs.device
    scaler = LossScaler(enabled=use_amp and amp_dtype == torch.float16 and dev.type == "cuda", device=dev)

    def step():
        optimizer.zero_grad(set_to_none=True)
        with torch.autocast(dev.type, dtype=amp_dtype, enabled=use_amp and dev.type == "cuda"):
            out = model(inputs)
            loss = criterion(out.float(), targets)
        if scaler.enabled:
            scaler.scale(loss).backward()
            scaler.step(optimizer)
            scaler.update()
        else:
            loss.backward()
            optimizer.step()

    for _ in range(warmup):
        step()
    _sync()
    if torch.cuda.is_available():
        torch.cuda.reset_peak_memory_stats()
    t0 = time.perf_counter()
    for _ in range(num_iterations):
        step()
    _sync()
    total = time.perf_counter() - t0
    avg = total / num_iterations
    mem = torch.cuda.max_memory_allocated() / 2**20 if torch.cuda.is_available() else 0.0
    return {"total_time": total, "avg_time": avg, "throughput": inputs.shape[0] / avg, "memory_usage": mem}


def compare_precision_formats(model_fn: Callable[[], nn.Module], input_shape: Sequence[int],
                              batch_sizes: Sequence[int] = (1, 2, 4, 8, 16, 32, 64), num_iterations: int = 20,
                              warmup: int = 5):
    """Cast the model to fp32 / fp16 / bf16 and sweep batch sizes (forward + training step)."""
    import pandas as pd

    dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    rows: List[Dict] = []
    for name, dt in (("fp32", torch.float32), ("fp16", torch.float16), ("bf16", torch.bfloat16)):
        if dev.type == "cpu" and dt == torch.float16:
            continue
        for b in batch_sizes:
            try:
                model = model_fn().to(dev).to(dt)
                x = torch.rand(b, *input_shape[1:], device=dev, dtype=dt)
                fwd = benchmark_forward_pass(model, x, num_iterations, warmup)
                out = model(x)
                y = torch.rand_like(out.float())
                opt = torch.optim.Adam(model.parameters(), lr=1e-3)
                tr = benchmark_training_step(model, x, y, opt, nn.MSELoss(), num_iterations, warmup)
                rows.append({"precision": name, "batch_size": b, "fwd_ms": fwd["avg_time"] * 1e3,
                             "fwd_throughput": fwd["throughput"], "train_ms": tr["avg_time"] * 1e3,
                             "train_throughput": tr["throughput"], "memory_mb": tr["memory_usage"]})
            except RuntimeError as e:
                print(f"{name} batch {b}: {e}")
                break
    return pd.DataFrame(rows)


def save_benchmark_results(results, filename: str, results_dir: str = "results/benchmarks") -> None:
    import pandas as pd

    os.makedirs(results_dir, exist_ok=True)
    df = results if isinstance(results, pd.DataFrame) else pd.DataFrame(results)
    path = os.path.join(results_dir, filename)
    if filename.endswith(".json"):
        df.to_json(path, orient="records", indent=2)
    else:
        df.to_csv(path, index=False)
    print(f"saved {path}")
