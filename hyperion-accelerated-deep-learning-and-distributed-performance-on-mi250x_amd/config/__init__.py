"""Typed configuration that is actually loaded (the reference's ``Phase 1/default_config.json`` had
no reader at all — SURVEY C10, §5.6).

Same four sections as that file (``hardware``, ``optimization``, ``benchmarking``,
``distributed``) plus ``training`` (the knobs the reference hard-coded inside each trainer).
``load_config(path)`` reads JSON or YAML (``yaml.safe_load`` only), validates keys against the
dataclasses (unknown keys are an error, not silently ignored), and ``apply_to_args`` overlays a
config onto the ``run_distributed`` argparse namespace (explicit CLI flags win).
Defaults are MI355X's, not MI250X's.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional


@dataclass
class HardwareConfig:
    gpu_type: str = "MI355X"
    arch: str = "gfx950"
    num_gpus: int = 8
    memory_per_gpu_gb: int = 288
    xgmi_links_per_gpu: int = 7
    xgmi_link_gbps: float = 153.0


@dataclass
class OptimizationConfig:
    enable_amp: bool = True
    amp_dtype: str = "bf16"
    amp_mode: str = "copies"              # copies (bf16 weights + fp32 masters) | autocast
    enable_compile: bool = False          # no Inductor/Triton on this stack; see enable_hipgraph
    compile_mode: str = "reduce-overhead"
    enable_hipgraph: bool = True          # the MI355X replacement for compile(mode="reduce-overhead")
    kernels: str = "hyperion"             # hyperion | torch
    optimize_dataloader: bool = True
    set_omp_threads: bool = True
    enable_channels_last: bool = True
    gradient_accumulation_steps: int = 1
    enable_gradient_checkpointing: bool = False
    distributed_strategy: str = "ddp"     # ddp | fsdp
    ddp_bucket_mb: float = 64.0
    fsdp_min_num_params: int = 100_000


@dataclass
class BenchmarkingConfig:
    batch_sizes: List[int] = field(default_factory=lambda: [1, 2, 4, 8, 16, 32, 64, 128])
    models: List[str] = field(default_factory=lambda: ["resnet50", "vit_b_16", "transformer"])
    precision_formats: List[str] = field(default_factory=lambda: ["fp32", "fp16", "bf16"])
    num_iterations: int = 50
    warmup_iterations: int = 10


@dataclass
class DistributedConfig:
    backend: str = "nccl"                 # = RCCL on ROCm
    init_method: str = "env://"
    timeout_s: float = 600.0
    master_addr: str = "127.0.0.1"


@dataclass
class TrainingConfig:
    epochs: int = 5
    seed: int = 0
    synthetic: bool = True
    precision: Optional[str] = None
    max_steps: Optional[int] = None
    dataset_size: Optional[int] = None
    ckpt_mode: str = "full"
    lora: bool = False
    lora_parallel: str = "fsdp"
    batch_size: int = 1


@dataclass
class HyperionConfig:
    hardware: HardwareConfig = field(default_factory=HardwareConfig)
    optimization: OptimizationConfig = field(default_factory=OptimizationConfig)
    benchmarking: BenchmarkingConfig = field(default_factory=BenchmarkingConfig)
    distributed: DistributedConfig = field(default_factory=DistributedConfig)
    training: TrainingConfig = field(default_factory=TrainingConfig)

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


def _build(cls, data: Dict[str, Any], where: str):
    names = {f.name: f for f in dataclasses.fields(cls)}
    unknown = set(data) - set(names)
    if unknown:
        raise ValueError(f"unknown key(s) in [{where}]: {sorted(unknown)}")
    kw = {}
    for k, v in data.items():
        f = names[k]
        if dataclasses.is_dataclass(f.default_factory() if f.default_factory is not dataclasses.MISSING else None):
            kw[k] = _build(type(f.default_factory()), v, f"{where}.{k}" if where else k)
        else:
            kw[k] = v
    return cls(**kw)


def from_dict(data: Dict[str, Any]) -> HyperionConfig:
    return _build(HyperionConfig, data, "")


def load_config(path: str) -> HyperionConfig:
    with open(path) as f:
        text = f.read()
    if path.endswith((".yaml", ".yml")):
        import yaml

        data = yaml.safe_load(text) or {}
    else:
        data = json.loads(text)
    return from_dict(data)


def save_config(cfg: HyperionConfig, path: str) -> None:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        json.dump(cfg.to_dict(), f, indent=2)


def apply_to_args(cfg: HyperionConfig, args, defaults: Optional[Dict[str, Any]] = None) -> None:
    """Fill argparse values that are still at their defaults from the config."""
    from ..cli.run_distributed import build_parser

    defaults = defaults or vars(build_parser().parse_args([]))
    t = cfg.training
    mapping = {"epochs": t.epochs, "seed": t.seed, "synthetic": t.synthetic, "precision": t.precision,
               "max_steps": t.max_steps, "dataset_size": t.dataset_size, "ckpt_mode": t.ckpt_mode, "lora": t.lora,
               "lora_parallel": t.lora_parallel, "batch_size": t.batch_size, "kernels": cfg.optimization.kernels}
    for k, v in mapping.items():
        if hasattr(args, k) and getattr(args, k) == defaults.get(k):
            setattr(args, k, v)
