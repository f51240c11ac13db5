"""Fused input BN + ReLU (conv_igemm.hip XF) vs apply pass + plain conv on the ResNet-50 consumer
shapes (batch 32, bf16, HBM-cold operands), with the XF parts switched off one at a time
(conv_set_xf_debug: 1 = no fragment transform, 2 = no inline finalize, 4 = no side store).

    python scripts/xf_bench.py [--out gpurun_out/xf_bench.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from conv_roofline import gtime_cold  # noqa: E402
from hyperion.ops import _native  # noqa: E402
from hyperion.ops.conv import _plan  # noqa: E402

# (name, N, C, H, K, R): the stride-1 consumers of a deferred BN in ResNet-50
SHAPES = [("l1_conv2", 32, 64, 56, 64, 3), ("l1_conv3", 32, 64, 56, 256, 1), ("l2_conv2", 32, 128, 28, 128, 3),
          ("l2_conv3", 32, 128, 28, 512, 1), ("l3_conv2", 32, 256, 14, 256, 3), ("l3_conv3", 32, 256, 14, 1024, 1),
          ("l4_conv2", 32, 512, 7, 512, 3), ("l4_conv3", 32, 512, 7, 2048, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/xf_bench.json")
    args = ap.parse_args()
    C = _native.native()
    S = _native.STAT_SLOTS
    rows = []
    for name, N, Cin, H, K, R in SHAPES:
        p = (R - 1) // 2
        y0 = (torch.randn(N, Cin, H, H, device="cuda")).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, Cin, R, R, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
        g, b = torch.ones(Cin, device="cuda"), torch.zeros(Cin, device="cuda")
        rm, rv = torch.zeros(Cin, device="cuda"), torch.ones(Cin, device="cuda")
        sums = torch.zeros(S, 2, Cin, device="cuda", dtype=torch.float64)
        sums[0, 0] = 0.0
        sums[0, 1] = float(N * H * H)
        sums = sums.reshape(-1)
        so = torch.zeros(S * 2 * K, device="cuda", dtype=torch.float64)
        xout = torch.empty_like(y0)
        st = torch.empty(2, Cin, device="cuda")
        pl = _plan("fwd", N * H * H, K, Cin, R, R, 1) or (-1, -1, -1, 0)
        r = {"name": name, "N": N, "C": Cin, "H": H, "K": K, "R": R, "plan": list(pl)}

        def plain():
            C.conv_fwd(y0, w, 1, 1, p, p, True, pl[0], pl[1], pl[2], sums=so, stages=pl[3])

        def apply():
            C.bn_fwd_sums(y0, None, sums, g, b, rm, rv, 0.1, 1e-5, True)

        def xf():
            C.conv_fwd(y0, w, 1, 1, p, p, True, pl[0], pl[1], pl[2], sums=so, stages=pl[3], xf_sums=sums, xf_w=g,
                       xf_b=b, xf_rm=rm, xf_rv=rv, xf_out=xout, xf_stats=st)

        r["plain_us"] = gtime_cold(plain)
        r["apply_us"] = gtime_cold(apply)
        for bits in (0, 1, 2, 4, 7):
            C.conv_set_xf_debug(bits)
            r[f"xf{bits}_us"] = gtime_cold(xf)
        C.conv_set_xf_debug(0)
        # tile alternatives for the fused kernel
        for bm, bn, nb in ((64, 64, 2), (128, 64, 2), (128, 128, 2), (64, 64, 1), (128, 64, 1)):
            if bn > K:
                continue

            def xft(bm=bm, bn=bn, nb=nb):
                C.conv_fwd(y0, w, 1, 1, p, p, True, bm, bn, 1, sums=so, stages=nb, xf_sums=sums, xf_w=g, xf_b=b,
                           xf_rm=rm, xf_rv=rv, xf_out=xout, xf_stats=st)

            r[f"xf_{bm}x{bn}_nb{nb}_us"] = gtime_cold(xft)
        print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        rows.append(r)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    json.dump(rows, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
