"""Fused-vs-eager benchmark — the MI355X replacement for the reference's torch.compile study (C32).

Reference (``02_development/compilation_optimization.py``): the 768-d LM (tokens ``[128, 8]``) and
ResNet-18 (CIFAR, batch 32, channels-last) in ``eval`` + ``no_grad``, variants "checkpoint"
(= eager), ``torch.compile(mode="default")`` and ``mode="max-autotune"``, 3 warm-up +
``--repeat`` iterations timed with wall clock, optional bf16 autocast; memory recorded as
``memory_allocated`` after the loop (not peak, polluted by earlier variants — SURVEY §5, BASELINE
§3).  Headline: ResNet-18 2.55 → 1.51 ms (1.68×), LM-768 5.99 → 5.60 ms (1.07×) on one MI250X GCD.

There is no Inductor/Triton here.  Variants:

* ``eager``       — PyTorch eager ops (``HYPERION_KERNELS=torch``): the reference's baseline;
* ``fused``       — Hyperion's gfx950 kernels (fused BN+ReLU(+residual) / LayerNorm(+residual) /
  flash attention / GEMM-epilogue activations), still one Python dispatch per op;
* ``fused_graph`` — the same, captured once into a hipGraph and replayed (the analogue of
  ``mode="reduce-overhead"``'s CUDA-graph trees).

Reported per variant: mean ms over ``repeat`` iterations (hipEvents), true PEAK memory of the
variant in isolation (reset before each), and the speedup vs eager.  CSV/JSON keep the reference
columns ``model,variant,time_ms,mem_gb`` (+ ``peak_mem_gb``, ``speedup``); also a TXT summary and
a PNG.
"""
from __future__ import annotations

import json
import os
from typing import Callable, Dict, List, Optional

import torch

from .baseline import _kernels


def _specs(batch_lm: int = 8, seq: int = 128, batch_cifar: int = 32):
    from ..models.resnet import resnet18
    from ..models.simple_lm import simple_lm_768

    def lm():
        return simple_lm_768()

    def lm_input(dev):
        return (torch.randint(0, 50257, (seq, batch_lm), device=dev),)

    def r18():
        return resnet18(num_classes=10)

    def r18_input(dev):
        return (torch.randn(batch_cifar, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last),)

    return [("simple_transformer_lm", lm, lm_input, False), ("resnet18_cifar10", r18, r18_input, True)]


def _time_variant(build: Callable, make_input: Callable, channels_last: bool, variant: str, dtype: Optional[torch.dtype],
                  repeat: int, warmup: int = 3) -> Dict:
    dev = torch.device("cuda")
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats()
    base_alloc = torch.cuda.memory_allocated()
    with _kernels("torch" if variant == "eager" else "hyperion"):
        model = build().to(dev).eval()
        if channels_last:
            model = model.to(memory_format=torch.channels_last)
        inputs = make_input(dev)

        def run():
            with torch.no_grad(), torch.autocast("cuda", dtype=dtype or torch.float32, enabled=dtype is not None):
                return model(*inputs)

        for _ in range(warmup):
            run()
        fn = run
        if variant == "fused_graph":
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                run()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                run()
            fn = g.replay
            for _ in range(warmup):
                fn()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(repeat):
            fn()
        en.record()
        en.synchronize()
        ms = st.elapsed_time(en) / repeat
    peak = (torch.cuda.max_memory_allocated() - base_alloc) / 1e9
    after = (torch.cuda.memory_allocated() - base_alloc) / 1e9
    return {"time_ms": ms, "peak_mem_gb": peak, "mem_gb": after}


def run_fusion_benchmark(base_dir: str = ".", dtype: str = "bf16", repeat: int = 10,
                         variants=("eager", "fused", "fused_graph")) -> List[Dict]:
    out_dir = os.path.join(base_dir, "results", "benchmarks", "compilation")
    os.makedirs(out_dir, exist_ok=True)
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": None}[dtype]
    rows = []
    for name, build, make_input, cl in _specs():
        eager_ms = None
        for v in variants:
            r = _time_variant(build, make_input, cl, v, dt, repeat)
            eager_ms = r["time_ms"] if v == "eager" else eager_ms
            r.update(model=name, variant=v, speedup=(eager_ms / r["time_ms"]) if eager_ms else None)
            rows.append(r)
            print(f"{name:22s} {v:12s} {r['time_ms']:8.3f} ms  peak {r['peak_mem_gb']:.3f} GB  "
                  f"x{(r['speedup'] or 1):.2f}")
    import pandas as pd

    df = pd.DataFrame(rows)[["model", "variant", "time_ms", "mem_gb", "peak_mem_gb", "speedup"]]
    df.to_csv(os.path.join(out_dir, "compilation_ckpt_benchmark.csv"), index=False)
    with open(os.path.join(out_dir, "compilation_ckpt_benchmark.json"), "w") as f:
        json.dump(rows, f, indent=2)
    with open(os.path.join(out_dir, "compilation_ckpt_analysis.txt"), "w") as f:
        for name in df.model.unique():
            sub = df[df.model == name]
            best = sub.loc[sub.time_ms.idxmin()]
            f.write(f"{name}: best {best.variant} {best.time_ms:.3f} ms ({best.speedup:.2f}x vs eager), "
                    f"peak {best.peak_mem_gb:.3f} GB\n")
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        fig, ax = plt.subplots(1, 2, figsize=(11, 4))
        for i, name in enumerate(df.model.unique()):
            sub = df[df.model == name]
            ax[0].bar([f"{name[:6]}\n{v}" for v in sub.variant], sub.time_ms)
            ax[1].bar([f"{name[:6]}\n{v}" for v in sub.variant], sub.peak_mem_gb)
        ax[0].set_ylabel("ms")
        ax[1].set_ylabel("peak GB")
        fig.tight_layout()
        fig.savefig(os.path.join(out_dir, "compilation_ckpt_speed_mem.png"), dpi=110)
        plt.close(fig)
    except Exception as e:  # pragma: no cover
        print(f"(plot skipped: {e})")
    return rows
