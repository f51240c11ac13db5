"""Hardware characterisation: matmul TFLOPS and STREAM bandwidth on raw HIP kernels.

Reference (``Phase 1/01_hardware_exploration.ipynb``):
* ``test_precision_formats`` (:208-242): square ``torch.matmul`` N ∈ {1024..8192} × {fp32, fp16,
  bf16}, TFLOPS = 2N³/t, with ONE un-warmed call whose timer also wraps both ``torch.rand``
  allocations (:223-231);
* ``test_memory_bandwidth`` (:263-301): one un-warmed fp32 ``z = x + y`` over {10..500}M elements,
  GB/s = 12n/t;
* ``test_gpu_operations`` (:171-205), ``get_gpu_memory`` (:161-164).

Hyperion runs each in two methodologies so the comparison is honest both ways:
``method='reference'`` reproduces the single-shot, allocation-inside-the-timer measurement;
``method='proper'`` warms up, times with hipEvents and reports the median of ``repeat`` runs.
Kernels: ``hyperion`` = the hand-written gfx950 GEMMs — bf16/fp16 on the deep-pipelined tiled MFMA
GEMM (``gemm_tiles.hip``; the proper method reports the best of its tile shapes, the reference
method the static plan), fp32 on the fp32-input MFMA GEMM (``gemm_f32.hip``: exact fp32 products,
no TF32-like shortcut exists on gfx950) — and the STREAM kernels (``stream_bw.hip``); ``torch`` =
hipBLASLt/rocBLAS and PyTorch's elementwise add, for A/B.
Results use the reference CSV schemas (``precision_results.csv``: ``Size,Precision,Time (s),TFLOPS``;
``bandwidth_results.csv``: ``Size (M elements),Bandwidth (GB/s)``) plus ``Method``/``Kernel`` columns.
"""
from __future__ import annotations

import os
import statistics
import time
from typing import Dict, List, Optional, Sequence

import torch

from ..utils.device import get_gpu_memory  # noqa: F401  (reference name, re-exported)

_DT = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def _events_ms(fn, repeat: int, warmup: int) -> List[float]:
    for _ in range(warmup):
        fn()
    out = []
    for _ in range(repeat):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        out.append(s.elapsed_time(e))
    return out


def matmul_tflops(n: int, precision: str, kernel: str = "hyperion", method: str = "proper", repeat: int = 20,
                  warmup: int = 5, tiles=(0, 1, 2, 3, 8, 9, 10, 11, 12)) -> Dict:
    """TFLOPS of one n×n×n product (2n³ FLOP).  Hyperion computes C = A·Bᵀ with B stored [N, K] (the
    transpose is layout, not work: same 2n³ FLOPs)."""
    from ..ops import _native

    dev = torch.device("cuda")
    dt = _DT[precision]
    use_hyp = kernel == "hyperion"
    C = _native.native() if use_hyp else None

    def make():
        a = torch.rand(n, n, device=dev, dtype=dt) * 2 - 1
        b = torch.rand(n, n, device=dev, dtype=dt) * 2 - 1
        return a, b

    def hyp_fn(a, b, tile=-1):
        if dt == torch.float32:
            return lambda: C.gemm_f32_nt(a, b)  # noqa: E731
        return lambda: C.gemm(a, b, tile=tile, splits=1 if tile >= 0 else -1)  # noqa: E731

    best_tile = None
    if method == "reference":
        _sync()
        t0 = time.perf_counter()
        a, b = make()  # allocation inside the timer, single un-warmed call (reference :223-231)
        c = hyp_fn(a, b)() if use_hyp else torch.matmul(a, b)
        _sync()
        t = time.perf_counter() - t0
        del c
    else:
        a, b = make()
        if use_hyp and dt != torch.float32:
            # the tiled kernel's tile shapes (the autotune space of ops/gemm.py): report the best
            res = {}
            for tile in tiles:
                try:
                    res[tile] = statistics.median(_events_ms(hyp_fn(a, b, tile), repeat, warmup)) / 1e3
                except RuntimeError:  # tile not valid for this shape
                    pass
            best_tile = min(res, key=res.get)
            t = res[best_tile]
        else:
            fn = hyp_fn(a, b) if use_hyp else (lambda: torch.matmul(a, b))  # noqa: E731
            t = statistics.median(_events_ms(fn, repeat, warmup)) / 1e3
    kname = "torch"
    if use_hyp:
        kname = "hyperion_f32_mfma" if dt == torch.float32 else "hyperion_tiled_mfma"
    return {"Size": n, "Precision": precision.upper() if precision != "bf16" else "BF16", "Time (s)": t,
            "TFLOPS": 2 * n**3 / t / 1e12, "Method": method, "Kernel": kname, "Tile": best_tile}


def test_precision_formats(sizes: Sequence[int] = (1024, 2048, 4096, 8192), precisions=("fp32", "fp16", "bf16"),
                           kernels=("hyperion", "torch"), methods=("proper", "reference"), results_dir: Optional[str] =
                           "results/benchmarks/hardware") -> List[Dict]:
    rows = []
    for method in methods:
        for kern in kernels:
            for p in precisions:
                for n in sizes:
                    r = matmul_tflops(n, p, kern, method)
                    rows.append(r)
                    print(f"{method:9s} {kern:8s} {p:5s} {n:5d}: {r['TFLOPS']:8.1f} TFLOPS ({r['Time (s)'] * 1e3:.3f} ms)")
    _save(rows, results_dir, "precision_results.csv")
    return rows


def stream_bandwidth(n: int, op: str = "add", kernel: str = "hyperion", method: str = "proper", repeat: int = 20,
                     warmup: int = 5, nontemporal: bool = True) -> Dict:
    """GB/s of a STREAM op over n fp32 elements (add/triad: 12n bytes; copy/scale: 8n)."""
    from ..ops import _native

    dev = torch.device("cuda")
    ops = {"copy": 0, "scale": 1, "add": 2, "triad": 3}
    nbytes = (12 if op in ("add", "triad") else 8) * n
    x = torch.rand(n, device=dev)
    y = torch.rand(n, device=dev)
    z = torch.empty(n, device=dev)
    if kernel == "hyperion":
        C = _native.native()
        fn = lambda: C.stream(ops[op], x, y if op in ("add", "triad") else None, z, 3.0, nontemporal, 0)  # noqa: E731
    else:
        fns = {"copy": lambda: z.copy_(x), "scale": lambda: torch.mul(x, 3.0, out=z),
               "add": lambda: torch.add(x, y, out=z), "triad": lambda: torch.add(x, y, alpha=3.0, out=z)}
        fn = fns[op]
    if method == "reference":
        _sync()
        t0 = time.perf_counter()
        fn()
        _sync()
        t = time.perf_counter() - t0
    else:
        t = statistics.median(_events_ms(fn, repeat, warmup)) / 1e3
    return {"Size (M elements)": n // 1_000_000 if n >= 1_000_000 else n / 1e6, "Bandwidth (GB/s)": nbytes / t / 1e9,
            "Op": op, "Method": method, "Kernel": kernel, "Time (s)": t}


def test_memory_bandwidth(sizes_m: Sequence[int] = (10, 20, 50, 100, 200, 500), ops=("add",),
                          kernels=("hyperion", "torch"), methods=("proper", "reference"),
                          results_dir: Optional[str] = "results/benchmarks/hardware") -> List[Dict]:
    rows = []
    for method in methods:
        for kern in kernels:
            for op in ops:
                for m in sizes_m:
                    r = stream_bandwidth(m * 1_000_000, op, kern, method)
                    rows.append(r)
                    print(f"{method:9s} {kern:8s} {op:5s} {m:4d}M: {r['Bandwidth (GB/s)']:8.1f} GB/s")
    _save(rows, results_dir, "bandwidth_results.csv")
    return rows


def test_gpu_operations() -> Dict[str, float]:
    """C2: rand 5000² ×2, one fp32 matmul 5000², and sin(x)+cos(y) — sync-bracketed wall times."""
    dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    out = {}
    _sync()
    t0 = time.perf_counter()
    x = torch.rand(5000, 5000, device=dev)
    y = torch.rand(5000, 5000, device=dev)
    _sync()
    out["rand_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    torch.matmul(x, y)
    _sync()
    out["matmul_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    torch.sin(x) + torch.cos(y)
    _sync()
    out["elementwise_s"] = time.perf_counter() - t0
    return out


def _save(rows: List[Dict], results_dir: Optional[str], name: str) -> None:
    if not results_dir or not rows:
        return
    import pandas as pd

    os.makedirs(results_dir, exist_ok=True)
    pd.DataFrame(rows).to_csv(os.path.join(results_dir, name), index=False)
    fn = {"precision_results.csv": "plot_precision_performance", "bandwidth_results.csv": "plot_memory_bandwidth"}.get(name)
    if fn:
        try:
            from . import plots

            getattr(plots, fn)(os.path.join(results_dir, name))
        except Exception as e:  # plotting is never fatal
            print(f"[plot] {fn} skipped: {e}")


test_precision_formats.__test__ = False  # reference names start with "test_"
test_memory_bandwidth.__test__ = False
test_gpu_operations.__test__ = False
