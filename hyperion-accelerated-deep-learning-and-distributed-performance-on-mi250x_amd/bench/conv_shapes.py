"""Per-layer convolution timing: Hyperion implicit-GEMM kernel vs the vendor (MIOpen) path.

Enumerates every distinct conv of ResNet-50 at a given batch (NHWC bf16), times forward with the
BN-statistics epilogue (ours) against ``F.conv2d`` (MIOpen, benchmark mode), and the stride-1
data gradient (ours: conv of dY with the flipped filter) against ``aten.convolution_backward``.
hipEvent timing, median of ``repeat``.  Drives the tile-selection heuristic in conv_igemm.hip.
"""
from __future__ import annotations

import statistics
from typing import Dict, List

import torch
import torch.nn.functional as F


def resnet50_convs(batch: int = 32) -> List[Dict]:
    from ..models.resnet import resnet50

    m = resnet50()
    shapes, seen = [], set()
    hw = {"conv1": 224}

    def visit(x_hw, conv):
        k = (conv.in_channels, x_hw, conv.out_channels, conv.kernel_size[0], conv.stride[0], conv.padding[0])
        if k not in seen:
            seen.add(k)
            shapes.append(dict(N=batch, C=k[0], H=k[1], K=k[2], R=k[3], stride=k[4], pad=k[5]))
        return (x_hw + 2 * conv.padding[0] - conv.kernel_size[0]) // conv.stride[0] + 1

    h = visit(hw["conv1"], m.conv1)
    h = (h + 2 - 3) // 2 + 1  # maxpool
    for layer in (m.layer1, m.layer2, m.layer3, m.layer4):
        for blk in layer:
            h1 = visit(h, blk.conv1)
            h2 = visit(h1, blk.conv2)
            visit(h2, blk.conv3)
            if blk.downsample is not None:
                visit(h, blk.downsample[0])
            h = h2
    return shapes


def _med(fn, repeat=20, warmup=5) -> float:
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(repeat):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return statistics.median(ts)


def run(batch: int = 32, sweep: bool = False) -> List[Dict]:
    from ..ops import _native

    torch.backends.cudnn.benchmark = True
    C_ = _native.native()
    rows = []
    for sh in resnet50_convs(batch):
        N, C, H, K, R, s, p = sh["N"], sh["C"], sh["H"], sh["K"], sh["R"], sh["stride"], sh["pad"]
        x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, C, R, R, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        P = (H + 2 * p - R) // s + 1
        flop = 2.0 * N * P * P * K * C * R * R
        r = dict(sh, P=P, gflop=flop / 1e9)
        r["miopen_fwd_us"] = _med(lambda: F.conv2d(x, w, stride=s, padding=p))
        if C % 64 == 0:
            r["hyp_fwd_us"] = _med(lambda: C_.conv_fwd(x, w, s, s, p, p, True))
        dy = torch.randn(N, K, P, P, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        r["miopen_dgrad_us"] = _med(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [True, False, False]))
        r["miopen_wgrad_us"] = _med(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [False, True, False]))
        if s == 1 and K % 64 == 0:
            r["hyp_dgrad_us"] = _med(lambda: C_.conv_dgrad(dy, w, p, p))
        if C % 64 == 0:
            r["hyp_wgrad_us"] = _med(lambda: C_.conv_wgrad(dy, x, R, R, s, s, p, p))
        if sweep:  # tile shapes of the fwd / dgrad kernels (automatic plan otherwise)
            for bm, bn in ((64, 64), (128, 64), (128, 128)):
                if C % 64 == 0:
                    r[f"hyp_fwd_{bm}x{bn}_us"] = _med(lambda: C_.conv_fwd(x, w, s, s, p, p, True, bm, bn), repeat=10)
                if s == 1 and K % 64 == 0:
                    r[f"hyp_dgrad_{bm}x{bn}_us"] = _med(lambda: C_.conv_dgrad(dy, w, p, p, bm, bn), repeat=10)
        for k in ("hyp_fwd_us", "miopen_fwd_us", "hyp_dgrad_us", "miopen_dgrad_us", "hyp_wgrad_us", "miopen_wgrad_us"):
            if k in r:
                r[k.replace("_us", "_tflops")] = flop / (r[k] * 1e-6) / 1e12
        rows.append(r)
        print({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}, flush=True)
    return rows
