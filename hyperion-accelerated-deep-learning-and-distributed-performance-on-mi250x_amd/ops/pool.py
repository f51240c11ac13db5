"""NHWC pooling on gfx950 (``csrc/kernels/pool.hip``): max pool and global average pool.

Reference: the ResNet stem ``nn.MaxPool2d(3, 2, 1)`` and head ``nn.AdaptiveAvgPool2d((1, 1))``
(torchvision ResNet via ``baseline_performance.ipynb:203-205``, ``distributed_utils.py:229``) and the
fallback CNN's two max pools (``baseline_performance.ipynb:226-236``); SURVEY §2.4 "Pooling".

* ``MaxPool2d`` — same module / constructor as ``nn.MaxPool2d``; on channels-last bf16/f16/f32
  GPU tensors (C % 8 == 0, no dilation, no ceil_mode) the forward records each element's winning
  window tap (uint8) and the backward is a deterministic gather (no atomics, no zero fill).
* ``AdaptiveAvgPool2d`` — output (1, 1) on channels-last GPU tensors runs the NHWC global-average
  kernels; anything else is PyTorch's.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, pad):
        y, idx = _native.native().maxpool2d_fwd(x, k, s, pad)
        ctx.save_for_backward(idx)
        ctx.cfg = (x.shape[2], x.shape[3], k, s, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        H, W, k, s, pad = ctx.cfg
        dx = _native.native().maxpool2d_bwd(dy.contiguous(memory_format=torch.channels_last), idx, H, W, k, s, pad)
        return dx, None, None, None


class _GapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        return _native.native().global_avgpool_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return _native.native().global_avgpool_bwd(dy.contiguous(), *ctx.hw)


def _nhwc_ok(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and x.shape[1] % 8 == 0 and x.is_contiguous(memory_format=torch.channels_last)
            and _native.use_native(x, op="pool"))


def max_pool2d(x: torch.Tensor, kernel_size, stride=None, padding=0) -> torch.Tensor:
    k, s, p = _pair(kernel_size), _pair(stride if stride is not None else kernel_size), _pair(padding)
    if _nhwc_ok(x) and k[0] == k[1] and s[0] == s[1] and p[0] == p[1] and p[0] < k[0] and k[0] * k[0] <= 256:
        return _native.apply_fn(_MaxPoolFn, x, k[0], s[0], p[0])
    return F.max_pool2d(x, k, s, p)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """``[N, C, H, W] -> [N, C, 1, 1]`` mean over H, W."""
    if _nhwc_ok(x):
        return _native.apply_fn(_GapFn, x).view(x.shape[0], x.shape[1], 1, 1)
    return F.adaptive_avg_pool2d(x, 1)


class MaxPool2d(nn.MaxPool2d):
    def forward(self, x: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        if self.dilation not in (1, (1, 1)) or self.ceil_mode or self.return_indices:
            return super().forward(x)
        return max_pool2d(x, self.kernel_size, self.stride, self.padding)


class AdaptiveAvgPool2d(nn.AdaptiveAvgPool2d):
    def forward(self, x: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        if _pair(self.output_size) == (1, 1):
            return global_avg_pool(x)
        return super().forward(x)
