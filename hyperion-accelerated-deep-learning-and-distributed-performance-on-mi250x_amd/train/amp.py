"""Mixed precision: bf16/fp16 compute copies with fp32 masters, and a device-side loss scaler.

Reference AMP: ``torch.cuda.amp.autocast()`` (fp16) + ``GradScaler`` in the
single-GPU and DDP trainers, ``MixedPrecision(bf16)`` for FSDP.  Two Hyperion modes:

* ``autocast`` — exactly the reference semantics (fp32 params, per-op casts);
* ``compute_copies`` — :func:`cast_for_compute` stores conv/linear/embedding weights in bf16 (or
  fp16) and keeps normalization parameters fp32; :class:`~hyperion.ops.optim.FusedAdam` keeps an
  fp32 master per low-precision parameter and rewrites the compute copy after each update.  This
  removes the per-forward weight casts and the per-backward grad casts autocast inserts (≈110
  small kernels per ResNet-50 step) — the O2-style recipe, done natively in the fused optimizer.

:class:`LossScaler` is a GradScaler equivalent whose scale / found-inf live on the device: the
unscale + inf-check is one multi-tensor kernel, and the optimizer skips the step on overflow by
reading the flag itself (no host sync, hipGraph-capturable).  Its state dict is the real scaler
state (the reference saved a freshly constructed scaler: ``mixed_precision.ipynb:278-279``).
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional

import torch
import torch.nn as nn

from ..ops import _native
from ..ops.multi_tensor import TableCache

_NORM_TYPES = (nn.modules.batchnorm._BatchNorm, nn.LayerNorm, nn.GroupNorm)


def cast_for_compute(model: nn.Module, dtype: torch.dtype = torch.bfloat16) -> nn.Module:
    """Cast every parameter/buffer except normalization layers (and RMSNorm weights) to ``dtype``."""
    keep32 = set()
    for m in model.modules():
        if isinstance(m, _NORM_TYPES) or type(m).__name__ in ("RMSNorm", "LlamaRMSNorm"):
            for p in m.parameters(recurse=False):
                keep32.add(id(p))
            for b in m.buffers(recurse=False):
                keep32.add(id(b))
    with torch.no_grad():
        for m in model.modules():
            for name, p in list(m.named_parameters(recurse=False)):
                if id(p) not in keep32 and p.is_floating_point():
                    p.data = p.data.to(dtype)
            for name, b in list(m.named_buffers(recurse=False)):
                if b is not None and id(b) not in keep32 and b.is_floating_point():
                    setattr(m, name, b.to(dtype))
    return model


class LossScaler:
    """Dynamic loss scaling with device-resident state (GradScaler semantics)."""

    def __init__(self, init_scale: float = 2.0**16, growth_factor: float = 2.0, backoff_factor: float = 0.5,
                 growth_interval: int = 2000, enabled: bool = True, device=None):
        self.enabled = enabled
        self.growth_factor = growth_factor
        self.backoff_factor = backoff_factor
        self.growth_interval = growth_interval
        dev = device or (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.scale_t = torch.full((), init_scale, dtype=torch.float32, device=dev)
        self.inv_scale_t = torch.full((), 1.0 / init_scale, dtype=torch.float32, device=dev)
        self.found_inf_t = torch.zeros((), dtype=torch.float32, device=dev)
        self.growth_tracker = torch.zeros((), dtype=torch.int32, device=dev)
        self._tables = TableCache()
        self._unscaled = False

    def scale(self, loss: torch.Tensor) -> torch.Tensor:
        if not self.enabled:
            return loss
        return loss * self.scale_t.to(loss.dtype)

    @torch.no_grad()
    def unscale_(self, optimizer: torch.optim.Optimizer) -> None:
        if not self.enabled or self._unscaled:
            return
        self._unscaled = True  # GradScaler semantics: one unscale per step (clip may call it early)
        self.found_inf_t.zero_()
        from ..ops.optim import grad_of

        grads = [gr for g in optimizer.param_groups for gr in (grad_of(p) for p in g["params"]) if gr is not None]
        if not grads:
            return
        by_dtype: Dict[torch.dtype, list] = {}
        for g in grads:
            by_dtype.setdefault(g.dtype, []).append(g)
        for dt, gs in by_dtype.items():
            if _native.use_native(gs[0], op="unscale") and all(g.is_contiguous() or g.dim() == 4 for g in gs):
                try:
                    tab = self._tables.get(f"unscale_{dt}", [gs])
                    _native.native().unscale_mt(tab.ptrs, tab.sizes, tab.blocks, tab.chunk, self.inv_scale_t,
                                                self.found_inf_t, _native.DTYPE_CODE[dt])
                    continue
                except ValueError:
                    pass
            torch._amp_foreach_non_finite_check_and_unscale_(gs, self.found_inf_t, self.inv_scale_t)

    def step(self, optimizer: torch.optim.Optimizer, *args, **kwargs):
        if not self.enabled:
            return optimizer.step(*args, **kwargs)
        self.unscale_(optimizer)
        if hasattr(optimizer, "found_inf") and hasattr(optimizer, "inv_scale"):
            # FusedAdam reads the flag on device and skips by itself; grads are already unscaled
            optimizer.found_inf = self.found_inf_t
            optimizer.inv_scale = None
            return optimizer.step(*args, **kwargs)
        if float(self.found_inf_t) == 0.0:  # host sync only for non-fused optimizers
            return optimizer.step(*args, **kwargs)
        return None

    @torch.no_grad()
    def update(self) -> None:
        if not self.enabled:
            return
        self._unscaled = False
        torch._amp_update_scale_(self.scale_t, self.growth_tracker, self.found_inf_t, self.growth_factor,
                                 self.backoff_factor, self.growth_interval)
        torch.reciprocal(self.scale_t, out=self.inv_scale_t)

    def get_scale(self) -> float:
        return float(self.scale_t)

    def state_dict(self) -> Dict:
        return {
            "scale": float(self.scale_t),
            "growth_factor": self.growth_factor,
            "backoff_factor": self.backoff_factor,
            "growth_interval": self.growth_interval,
            "_growth_tracker": int(self.growth_tracker),
        }

    def load_state_dict(self, sd: Dict) -> None:
        self.scale_t.fill_(sd["scale"])
        self.inv_scale_t.fill_(1.0 / sd["scale"])
        self.growth_factor = sd.get("growth_factor", self.growth_factor)
        self.backoff_factor = sd.get("backoff_factor", self.backoff_factor)
        self.growth_interval = sd.get("growth_interval", self.growth_interval)
        self.growth_tracker.fill_(sd.get("_growth_tracker", 0))


def autocast(device_type: str = "cuda", dtype: Optional[torch.dtype] = torch.float16, enabled: bool = True):
    """Non-deprecated autocast (reference used ``torch.cuda.amp.autocast()``)."""
    if device_type == "cuda" and not torch.cuda.is_available():
        device_type = "cpu"
        if dtype == torch.float16:
            dtype = torch.bfloat16
    return torch.autocast(device_type=device_type, dtype=dtype, enabled=enabled and dtype is not None)


def parameters_dtype(params: Iterable[torch.Tensor]) -> Dict[torch.dtype, int]:
    out: Dict[torch.dtype, int] = {}
    for p in params:
        out[p.dtype] = out.get(p.dtype, 0) + p.numel()
    return out
