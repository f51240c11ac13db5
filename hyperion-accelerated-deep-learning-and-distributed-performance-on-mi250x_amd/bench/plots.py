"""The reference's result plots, from the CSVs this framework writes (reference schemas).

* ``visualize_baseline_results`` — 2x2 bars of fwd / bwd / opt / total ms, memory and throughput per
  model (``baseline_performance.ipynb:418-470``, ``model_benchmarks.csv``).
* ``visualize_batch_scaling`` — step time, throughput and "scaling efficiency" vs batch
  (``:532-582``, ``*_batch_scaling.csv``; efficiency = throughput(b) / (b · throughput(1)), as there).
* ``plot_precision_performance`` / ``plot_memory_bandwidth`` — the hardware notebook's
  ``precision_performance.png`` (TFLOPS vs size per precision) and ``memory_bandwidth.png``
  (``01_hardware_exploration.ipynb:248-260, 306-313``).

matplotlib runs headless (Agg); every function returns the PNG path.
"""
from __future__ import annotations

import os
from typing import Optional

import pandas as pd


def _plt():
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    return plt


def visualize_baseline_results(csv_path: str, out_png: Optional[str] = None) -> str:
    plt = _plt()
    df = pd.read_csv(csv_path)
    fig, ax = plt.subplots(2, 2, figsize=(12, 9))
    parts = ["Forward Time (ms)", "Backward Time (ms)", "Optimizer Time (ms)"]
    bottom = None
    for p in parts:
        ax[0, 0].bar(df["Model"], df[p], bottom=bottom, label=p.replace(" (ms)", ""))
        bottom = df[p] if bottom is None else bottom + df[p]
    ax[0, 0].set_title("Step breakdown (ms)")
    ax[0, 0].legend()
    ax[0, 1].bar(df["Model"], df["Total Time (ms)"], color="tab:purple")
    ax[0, 1].set_title("Total step time (ms)")
    ax[1, 0].bar(df["Model"], df["Memory Usage (MB)"], color="tab:green")
    ax[1, 0].set_title("Peak memory (MB)")
    ax[1, 1].bar(df["Model"], df["Throughput (samples/s)"], color="tab:orange")
    ax[1, 1].set_title("Throughput (samples/s)")
    for a in ax.flat:
        a.tick_params(axis="x", rotation=20)
    fig.tight_layout()
    out = out_png or os.path.splitext(csv_path)[0] + ".png"
    fig.savefig(out, dpi=110)
    plt.close(fig)
    return out


def visualize_batch_scaling(csv_path: str, out_png: Optional[str] = None) -> str:
    plt = _plt()
    df = pd.read_csv(csv_path).sort_values("Batch Size")
    b = df["Batch Size"].astype(float)
    thr = df["Throughput (samples/s)"].astype(float)
    eff = thr / (b * float(thr.iloc[0] / b.iloc[0]))
    fig, ax = plt.subplots(1, 3, figsize=(15, 4.5))
    ax[0].plot(b, df["Total Time (ms)"], "o-")
    ax[0].set_title("Step time (ms)")
    ax[1].plot(b, thr, "o-", color="tab:orange")
    ax[1].set_title("Throughput (samples/s)")
    ax[2].plot(b, eff, "o-", color="tab:green")
    ax[2].axhline(1.0, ls="--", color="gray")
    ax[2].set_title("Scaling efficiency vs linear-in-batch")
    for a in ax:
        a.set_xscale("log", base=2)
        a.set_xlabel("batch size")
    fig.tight_layout()
    out = out_png or os.path.splitext(csv_path)[0] + ".png"
    fig.savefig(out, dpi=110)
    plt.close(fig)
    return out


def plot_precision_performance(csv_path: str, out_png: Optional[str] = None) -> str:
    plt = _plt()
    df = pd.read_csv(csv_path)
    fig, ax = plt.subplots(figsize=(8, 5))
    keys = [c for c in ("Method", "Kernel") if c in df.columns]
    for name, g in df.groupby(["Precision"] + keys):
        label = " / ".join(str(v) for v in (name if isinstance(name, tuple) else (name,)))
        ax.plot(g["Size"], g["TFLOPS"], "o-", label=label)
    ax.set_xscale("log", base=2)
    ax.set_xlabel("matrix size N (N x N)")
    ax.set_ylabel("TFLOPS")
    ax.set_title("Matmul throughput by precision")
    ax.legend(fontsize=7)
    fig.tight_layout()
    out = out_png or os.path.join(os.path.dirname(csv_path), "precision_performance.png")
    fig.savefig(out, dpi=110)
    plt.close(fig)
    return out


def plot_memory_bandwidth(csv_path: str, out_png: Optional[str] = None) -> str:
    plt = _plt()
    df = pd.read_csv(csv_path)
    fig, ax = plt.subplots(figsize=(8, 5))
    keys = [c for c in ("Method", "Kernel") if c in df.columns]
    groups = df.groupby(keys) if keys else [("", df)]
    for name, g in groups:
        label = " / ".join(str(v) for v in (name if isinstance(name, tuple) else (name,))) or "add"
        ax.plot(g["Size (M elements)"], g["Bandwidth (GB/s)"], "o-", label=label)
    ax.set_xscale("log")
    ax.set_xlabel("vector size (M elements)")
    ax.set_ylabel("GB/s")
    ax.set_title("Memory bandwidth (z = x + y)")
    ax.legend(fontsize=7)
    fig.tight_layout()
    out = out_png or os.path.join(os.path.dirname(csv_path), "memory_bandwidth.png")
    fig.savefig(out, dpi=110)
    plt.close(fig)
    return out
