"""Activation checkpointing with the reference's API shapes.

Reference: ``SimpleTransformerLM(use_checkpoint=True)`` runs
``checkpoint_sequential(self.transformer.layers, n_layers, x)`` and ``checkpoint_resnet_blocks``
monkey-patches a torchvision ResNet-18's forward to checkpoint ``layer1..layer4``
(``memory_optimization.ipynb:194-262``).  Both used the deprecated reentrant default; here it is
``use_reentrant=False`` and per-segment, so recomputation works with the fused BN / LN kernels and
under FSDP (units re-gather before their recompute).
"""
from __future__ import annotations

import types

import torch
import torch.nn as nn
from torch.utils.checkpoint import checkpoint, checkpoint_sequential


def checkpoint_resnet_blocks(model: nn.Module, segments: int = 4) -> nn.Module:
    """Stem eager, ``layer1..layer4`` checkpointed, then avgpool/fc (in place; returns the model)."""
    stages = nn.Sequential(model.layer1, model.layer2, model.layer3, model.layer4)

    def forward_with_ckpt(self, x):
        x = self.maxpool(self.bn1(self.conv1(x))) if not hasattr(self, "relu") else \
            self.maxpool(self.relu(self.bn1(self.conv1(x))))
        if self.training and torch.is_grad_enabled():
            x = checkpoint_sequential(stages, segments, x, use_reentrant=False)
        else:
            x = stages(x)
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)

    model.forward = types.MethodType(forward_with_ckpt, model)
    model._ckpt_stages = stages  # keep a handle (not registered twice: Sequential holds references)
    return model


def checkpoint_module(module: nn.Module) -> nn.Module:
    """Wrap any module so its forward is recomputed in backward."""
    fwd = module.forward

    def forward(*args, **kwargs):
        if module.training and torch.is_grad_enabled():
            return checkpoint(fwd, *args, use_reentrant=False, **kwargs)
        return fwd(*args, **kwargs)

    module.forward = forward
    return module
