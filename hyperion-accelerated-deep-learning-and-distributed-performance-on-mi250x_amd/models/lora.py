"""LoRA adapters with PEFT-compatible module layout and adapter files (no ``peft`` dependency).

Reference: ``get_peft_model(model, LoraConfig(r=16, lora_alpha=32, lora_dropout=0.05,
target_modules=["q_proj","k_proj","v_proj","o_proj"], bias="none", task_type="CAUSAL_LM"))`` on
bf16 Llama-2-7B, then DDP; ``save_pretrained`` writes the adapter directory
(``02_development/distributed_utils.py:463-476,552``; SURVEY C26, §2.2 "PEFT/LoRA").

``LoRALinear`` keeps PEFT's attribute names (``base_layer``, ``lora_A.default``,
``lora_B.default``), so ``state_dict`` keys match a PEFT model's and ``save_adapter`` writes the
same ``adapter_model.safetensors`` / ``adapter_config.json`` pair (keys without the adapter name,
prefixed ``base_model.model.``) that ``PeftModel.from_pretrained`` reads.

Compute: ``y = x Wᵀ (+ b) + s · (drop(x) Aᵀ) Bᵀ`` through ``ops.lora.lora_linear`` — the frozen
base GEMM plus the low-rank update with the dropout mask regenerated from a seed in backward
(never stored), and no gradient buffer ever allocated for W.
"""
from __future__ import annotations

import json
import math
import os
from typing import Dict, Iterable, List

import torch
import torch.nn as nn

from ..ops.lora import lora_linear


class LoRALinear(nn.Module):
    def __init__(self, base: nn.Linear, r: int = 16, alpha: float = 32.0, dropout: float = 0.05,
                 adapter: str = "default"):
        super().__init__()
        self.base_layer = base
        self.in_features, self.out_features = base.in_features, base.out_features
        self.r = r
        self.lora_alpha = alpha
        self.scaling = {adapter: alpha / r}
        self.adapter = adapter
        dev, dt = base.weight.device, base.weight.dtype
        self.lora_A = nn.ModuleDict({adapter: nn.Linear(base.in_features, r, bias=False, device=dev, dtype=dt)})
        self.lora_B = nn.ModuleDict({adapter: nn.Linear(r, base.out_features, bias=False, device=dev, dtype=dt)})
        self.lora_dropout = nn.ModuleDict({adapter: nn.Dropout(dropout) if dropout > 0 else nn.Identity()})
        self.p = dropout
        nn.init.kaiming_uniform_(self.lora_A[adapter].weight, a=math.sqrt(5))
        nn.init.zeros_(self.lora_B[adapter].weight)
        base.weight.requires_grad_(False)
        if base.bias is not None:
            base.bias.requires_grad_(False)

    @property
    def weight(self) -> torch.Tensor:  # code that reads q_proj.weight keeps working
        return self.base_layer.weight

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        a = self.adapter
        p = self.p if self.training else 0.0
        return lora_linear(x, self.base_layer.weight, self.base_layer.bias, self.lora_A[a].weight,
                           self.lora_B[a].weight, self.scaling[a], p)

    @torch.no_grad()
    def merged_weight(self) -> torch.Tensor:
        a = self.adapter
        dw = (self.lora_B[a].weight.float() @ self.lora_A[a].weight.float()) * self.scaling[a]
        return (self.base_layer.weight.float() + dw).to(self.base_layer.weight.dtype)


def apply_lora(model: nn.Module, r: int = 16, alpha: float = 32.0, dropout: float = 0.05,
               target_modules: Iterable[str] = ("q_proj", "k_proj", "v_proj", "o_proj"),
               adapter: str = "default") -> nn.Module:
    """Freeze every parameter and wrap target ``nn.Linear``s in :class:`LoRALinear` (in place)."""
    targets = set(target_modules)
    for p in model.parameters():
        p.requires_grad_(False)
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            if cname in targets and isinstance(child, nn.Linear) and not isinstance(child, LoRALinear):
                setattr(mod, cname, LoRALinear(child, r, alpha, dropout, adapter))
    model.peft_config = {adapter: lora_config_dict(r, alpha, dropout, sorted(targets))}
    return model


def lora_config_dict(r: int, alpha: float, dropout: float, targets: List[str],
                     base_model: str = "NousResearch/Llama-2-7b-hf") -> Dict:
    return {
        "peft_type": "LORA",
        "task_type": "CAUSAL_LM",
        "r": r,
        "lora_alpha": alpha,
        "lora_dropout": dropout,
        "target_modules": targets,
        "bias": "none",
        "fan_in_fan_out": False,
        "inference_mode": False,
        "base_model_name_or_path": base_model,
    }


def lora_state_dict(model: nn.Module, adapter: str = "default", prefix: str = "base_model.model.") -> Dict[str, torch.Tensor]:
    """PEFT adapter keys: ``base_model.model.<path>.lora_A.weight`` (adapter name stripped)."""
    out = {}
    for name, t in model.state_dict().items():
        if ".lora_A." in name or ".lora_B." in name:
            out[prefix + name.replace(f".{adapter}.", ".")] = t.detach().cpu().contiguous()
    return out


def save_adapter(model: nn.Module, out_dir: str, adapter: str = "default") -> str:
    """``save_pretrained`` equivalent: ``adapter_model.safetensors`` + ``adapter_config.json``."""
    from safetensors.torch import save_file

    os.makedirs(out_dir, exist_ok=True)
    save_file(lora_state_dict(model, adapter), os.path.join(out_dir, "adapter_model.safetensors"))
    cfg = getattr(model, "peft_config", {}).get(adapter) or lora_config_dict(16, 32, 0.05, ["q_proj", "k_proj", "v_proj", "o_proj"])
    with open(os.path.join(out_dir, "adapter_config.json"), "w") as f:
        json.dump(cfg, f, indent=2)
    return out_dir


def load_adapter(model: nn.Module, in_dir: str, adapter: str = "default", prefix: str = "base_model.model.") -> None:
    from safetensors.torch import load_file

    sd = load_file(os.path.join(in_dir, "adapter_model.safetensors"))
    own = model.state_dict()
    with torch.no_grad():
        for k, v in sd.items():
            name = k[len(prefix):] if k.startswith(prefix) else k
            name = name.replace(".lora_A.", f".lora_A.{adapter}.").replace(".lora_B.", f".lora_B.{adapter}.")
            own[name].copy_(v.to(own[name].dtype))


def trainable_parameters(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def merge_lora(model: nn.Module) -> nn.Module:
    """Fold every adapter into its base weight and unwrap (inference export)."""
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            if isinstance(child, LoRALinear):
                base = child.base_layer
                base.weight.data.copy_(child.merged_weight())
                setattr(mod, cname, base)
    return model

