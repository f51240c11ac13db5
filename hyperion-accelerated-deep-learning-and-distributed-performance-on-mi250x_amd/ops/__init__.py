"""Autograd ops over the hand-written gfx950 kernels in ``hyperion._C``.

Every op has a PyTorch reference implementation (CPU path and numerics oracle); the native path
runs on GPU tensors and fails loudly if the extension is missing (see ``_native``).
"""
from . import _native  # noqa: F401
from .batchnorm import BatchNormAct1d, BatchNormAct2d, bn_act  # noqa: F401
from .optim import FusedAdam, FusedAdamW, clip_grad_norm_  # noqa: F401
