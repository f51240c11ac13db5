"""CLI: the model benchmark suite on one GPU → ``results/benchmarks/models/*.json|csv``.

Runs the baseline step benchmark in the reference methodology (fp32, torch kernels) and in the
MI355X configuration (bf16 + Hyperion kernels), ResNet-50 batch scaling, the LM / ViT / Llama
step benchmarks and the fused-vs-eager study.  ``--only`` selects parts.
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--out", default="results/benchmarks/models")
    ap.add_argument("--only", default="baseline,scaling,lm,vit,llama,fsdp,fusion")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args(argv)
    parts = set(a.only.split(","))
    os.makedirs(a.out, exist_ok=True)
    summary = {}

    def dump():
        with open(os.path.join(a.out, "summary.json"), "w") as f:
            json.dump(summary, f, indent=2)

    if "baseline" in parts:
        from hyperion.bench.baseline import run_baseline_benchmarks

        summary["baseline_fp32_torch"] = run_baseline_benchmarks(a.out, "fp32", "torch", a.iters, 5,
                                                                 out_name="model_benchmarks_fp32_torch.csv")
        summary["baseline_fp32_hyperion"] = run_baseline_benchmarks(a.out, "fp32", "hyperion", a.iters, 5,
                                                                    out_name="model_benchmarks_fp32_hyperion.csv")
        summary["baseline_bf16_hyperion"] = run_baseline_benchmarks(a.out, "bf16", "hyperion", a.iters, 5,
                                                                    out_name="model_benchmarks_bf16_hyperion.csv")
        dump()
    if "scaling" in parts:
        from hyperion.bench.baseline import test_batch_size_scaling
        from hyperion.models.resnet import create_resnet50

        summary["resnet50_batch_scaling_bf16"] = test_batch_size_scaling(
            create_resnet50, lambda b: (b, 3, 224, 224), lambda b: (b, 1000), (1, 2, 4, 8, 16, 32, 64, 128, 256),
            a.iters, 5, "bf16", "hyperion", a.out)
        dump()
    if "lm" in parts:
        from hyperion.bench.models import bench_lm_step

        summary["lm256_fp16"] = bench_lm_step(precision="fp16")
        summary["lm256_bf16"] = bench_lm_step(precision="bf16")
        summary["lm256_bf16_graph"] = bench_lm_step(precision="bf16", graph=True)
        summary["gpt2_small_bf16_graph"] = bench_lm_step(precision="bf16", graph=True, model="gpt2_small", batch=16)
        print(summary["lm256_fp16"], summary["lm256_bf16"], summary["lm256_bf16_graph"],
              summary["gpt2_small_bf16_graph"], flush=True)
        dump()
    if "vit" in parts:
        from hyperion.bench.models import bench_vit_step

        summary["vit_b16_bf16_ckpt"] = bench_vit_step(checkpointing=True)
        summary["vit_b16_bf16_ckpt_graph"] = bench_vit_step(checkpointing=True, graph=True)
        summary["vit_b16_bf16"] = bench_vit_step(checkpointing=False)
        summary["vit_b16_bf16_graph"] = bench_vit_step(checkpointing=False, graph=True)
        print(summary["vit_b16_bf16_ckpt"], summary["vit_b16_bf16_ckpt_graph"], summary["vit_b16_bf16"],
              summary["vit_b16_bf16_graph"], flush=True)
        dump()
    if "llama" in parts:
        from hyperion.bench.models import bench_llama_lora_step

        summary["llama7b_lora_bf16_graph"] = bench_llama_lora_step(graph=True)
        summary["llama7b_lora_bf16_eager"] = bench_llama_lora_step(graph=False)
        print(summary["llama7b_lora_bf16_graph"], summary["llama7b_lora_bf16_eager"], flush=True)
        dump()
    if "fsdp" in parts:
        from hyperion.bench.models import bench_fsdp_step

        for name, kw in (("lm256", {}), ("gpt2_small", {"batch": 16}), ("llama7b_lora", {"batch": 1, "steps": 5})):
            summary[f"fsdp_{name}_bf16"] = bench_fsdp_step(name, **kw)
            print(summary[f"fsdp_{name}_bf16"], flush=True)
            dump()
    if "fusion" in parts:
        from hyperion.bench.fusion import run_fusion_benchmark

        summary["fusion"] = run_fusion_benchmark(os.path.dirname(a.out) or ".", "bf16", 20)
        dump()
    return 0


if __name__ == "__main__":
    sys.exit(main())
