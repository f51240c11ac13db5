"""ResNet-18 / ResNet-50 with torchvision-compatible state-dict keys.

Reference users: ``create_resnet50`` (``Phase 1/baseline_performance.ipynb:203-205``, via torch.hub),
torchvision ``resnet18(num_classes=10)`` in ``02_development/distributed_utils.py:229`` and
``compilation_optimization.py:82-93``.  torchvision is not a dependency here, so the networks are
defined from scratch.

MI355X design: every ``conv -> BN -> ReLU`` (and the bottleneck tail ``conv -> BN -> +identity
-> ReLU``) is expressed as ``conv`` followed by one ``BatchNormAct2d`` module, which dispatches to
the fused NHWC HIP kernels in ``hyperion.ops.batchnorm`` (stats pass + one apply pass with the
residual add and ReLU folded in; fused backward).  Module attribute names (``conv1``, ``bn1``,
``layer1.0.downsample.1`` …) match torchvision so checkpoints interchange.
"""
from __future__ import annotations

import os
from typing import List, Optional, Type, Union

import torch
import torch.nn as nn

from ..ops import _native
from ..ops.pool import AdaptiveAvgPool2d, MaxPool2d

from ..ops.batchnorm import BatchNormAct2d
from ..ops.conv_f32 import Conv2d
from ..ops.conv import branch_sum_link, conv_bn_act, residual_link, xf_consumer_ok
from ..ops.linear import Linear


def _downsample(ds: nn.Sequential, x: torch.Tensor, branch=None) -> torch.Tensor:
    """``downsample = Sequential(conv1x1, BatchNormAct2d)`` (torchvision keys ``downsample.0/1``)."""
    return conv_bn_act(ds[0], ds[1], x, branch=branch)


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return Conv2d(cin, cout, 1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = BatchNormAct2d(planes, act=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = BatchNormAct2d(planes, act=True)  # act applied after the residual add
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # identity shortcut: its gradient goes to conv1's dgrad store; downsample: the two data
        # gradients of x (downsample, conv1) are summed in-kernel
        branch = branch_sum_link(x) if self.downsample is not None else None
        identity = x if self.downsample is None else _downsample(self.downsample, x, branch)
        link = residual_link(x) if self.downsample is None else None
        # bn1 + ReLU applied by conv2's operand read (no apply pass) where conv2 can take it
        out = conv_bn_act(self.conv1, self.bn1, x, link=link, branch=branch, defer=xf_consumer_ok(self.conv2))
        return conv_bn_act(self.conv2, self.bn2, out, residual=identity, link=link)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None):
        super().__init__()
        width = planes
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = BatchNormAct2d(width, act=True)
        self.conv2 = conv3x3(width, width, stride)  # torchvision v1.5: stride on the 3x3
        self.bn2 = BatchNormAct2d(width, act=True)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = BatchNormAct2d(planes * self.expansion, act=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # identity shortcut: its gradient goes to conv1's dgrad store; downsample: the two data
        # gradients of x (downsample, conv1) are summed in-kernel
        branch = branch_sum_link(x) if self.downsample is not None else None
        identity = x if self.downsample is None else _downsample(self.downsample, x, branch)
        link = residual_link(x) if self.downsample is None else None
        # bn1 / bn2 + ReLU applied by the next conv's operand read (no apply passes) where it can
        out = conv_bn_act(self.conv1, self.bn1, x, link=link, branch=branch, defer=xf_consumer_ok(self.conv2))
        out = conv_bn_act(self.conv2, self.bn2, out, defer=xf_consumer_ok(self.conv3))
        return conv_bn_act(self.conv3, self.bn3, out, residual=identity, link=link)


class ResNet(nn.Module):
    def __init__(
        self,
        block: Type[Union[BasicBlock, Bottleneck]],
        layers: List[int],
        num_classes: int = 1000,
        zero_init_residual: bool = False,
    ):
        super().__init__()
        self.inplanes = 64
        self.conv1 = Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = BatchNormAct2d(64, act=True)
        self.maxpool = MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = AdaptiveAvgPool2d((1, 1))
        # (Hyperion's Linear measured slower here: 3 native launches for the [32, 2048] x 1000 head
        # vs hipBLASLt's one — HYPERION_RESNET_FC=native opts in)
        fc_cls = Linear if os.environ.get("HYPERION_RESNET_FC", "torch") == "native" else nn.Linear
        self.fc = fc_cls(512 * block.expansion, num_classes)
        # head_in_loss: forward returns the pooled features and the loss applies fc
        # (ops.losses.LinearMSELoss: the fused classifier + MSE of the step benchmark)
        self.head_in_loss = False

        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _make_layer(self, block, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                conv1x1(self.inplanes, planes * block.expansion, stride),
                BatchNormAct2d(planes * block.expansion, act=False),
            )
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward_features(self, x: torch.Tensor) -> torch.Tensor:
        x = self.maxpool(conv_bn_act(self.conv1, self.bn1, x))
        x = self.layer1(x)
        x = self.layer2(x)
        x = self.layer3(x)
        return self.layer4(x)

    # Each forward (or graph stage) opens one zero_scope: every BN statistics accumulator of the
    # pass is a slice of one buffer zeroed by a single fill (ops/_native.py ZeroArena).
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        with _native.zero_scope(self, "forward", x.device):
            x = self.forward_features(x)
            x = torch.flatten(self.avgpool(x), 1)
            return x if self.head_in_loss else self.fc(x)

    def _bottom(self, x: torch.Tensor) -> torch.Tensor:
        with _native.zero_scope(self, "bottom", x.device):
            return self.layer1(self.maxpool(conv_bn_act(self.conv1, self.bn1, x)))

    def _top(self, h: torch.Tensor) -> torch.Tensor:
        with _native.zero_scope(self, "top", h.device):
            x = self.layer4(self.layer3(self.layer2(h)))
            x = torch.flatten(self.avgpool(x), 1)
            return x if self.head_in_loss else self.fc(x)

    def graph_stages(self):
        """``forward(x) == top(bottom(x))``, cut after layer1: 99% of the gradient bytes (layer2-4,
        fc) are above the cut, while the bottom's backward (stem + the 56x56 layer1, ~1/4 of the
        backward time) is long enough to hide their all-reduce — the data-parallel hipGraph step
        (``train/step.py``) reduces the top buckets on the comm stream while it replays."""
        return [self._bottom, self._top]

    def graph_stage_modules(self):
        """Modules of each ``graph_stages`` stage (DDP starts a new gradient bucket at the cut)."""
        return [[self.conv1, self.bn1, self.layer1], [self.layer2, self.layer3, self.layer4, self.fc]]


def resnet18(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes=num_classes, **kw)


def resnet34(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes=num_classes, **kw)


def resnet50(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes=num_classes, **kw)


def create_resnet50() -> ResNet:
    """Reference-name factory (``baseline_performance.ipynb:203-205``)."""
    return resnet50(num_classes=1000)
