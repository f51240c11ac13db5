"""Per-shape launch-plan tuning of the native conv kernels (the MIOpen find-db role) on every
ResNet-50 convolution at a given batch: forward with the BN-statistics epilogue, the data
gradient with the producer's BN-backward epilogue (mode 1, the common case in a bottleneck) and
without it (the block-input convs), and the weight gradient — tile (bm x bn), split-K count and
(fwd / dgrad) LDS ring depth, each timed as 20 launches in one hipGraph.

Writes the winners to configs/conv_plans_mi355x.json (ops/conv.py looks plans up by GEMM shape)
and every measurement to gpurun_out/conv_tune.json.

    python scripts/conv_tune.py [--batch 32] [--out configs/conv_plans_mi355x.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.bench.conv_shapes import resnet50_convs  # noqa: E402
from hyperion.ops import _native  # noqa: E402
from conv_roofline import gtime as _gtime_warm, gtime_cold  # noqa: E402

gtime = gtime_cold  # plans are chosen on HBM-cold operands (--warm: repeat-loop timing)

TILES = [(128, 128), (128, 64), (64, 64)]


def configs(nk, strided_dgrad=False):
    out = []
    for bm, bn in TILES:
        for sp in ([1] if strided_dgrad else [1, 2, 3, 4, 6]):
            if sp > 1 and nk // sp < 2:
                continue
            for nb in (1, 2, 3):
                if nb == 3 and nk // sp < 6:
                    continue
                out.append((bm, bn, sp, nb))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--out", default="configs/conv_plans_mi355x.json")
    ap.add_argument("--raw", default="gpurun_out/conv_tune.json")
    ap.add_argument("--warm", action="store_true", help="time repeat loops (operands cache-resident)")
    ap.add_argument("--dual", action="store_true",
                    help="time every data-gradient plan INSIDE the fused data + weight gradient launch "
                         "(conv_dgrad_wgrad, what the training step runs): no dgrad split-K there")
    a = ap.parse_args()
    global gtime
    if a.warm:
        gtime = _gtime_warm
    C_ = _native.native()
    plans, raw = [], []
    for sh in resnet50_convs(a.batch):
        N, C, H, K, R, s, p = sh["N"], sh["C"], sh["H"], sh["K"], sh["R"], sh["stride"], sh["pad"]
        if C % 64:
            continue
        P = (H + 2 * p - R) // s + 1
        x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, C, R, R, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
        sums = torch.zeros(_native.STAT_SLOTS * 2 * K, device="cuda", dtype=torch.float64)
        row = dict(sh, P=P)
        # ---- forward + BN statistics
        nk = R * R * C // 64
        fwd = {}
        for cfg in configs(nk) + [(bm, bn, 1, nb + 16) for (bm, bn, sp, nb) in configs(nk) if sp == 1]:
            bm, bn, sp, nb = cfg  # (nb + 16: the DIRECT store epilogue)
            fwd[cfg] = gtime(lambda: C_.conv_fwd(x, w, s, s, p, p, True, bm, bn, sp, sums=sums, stages=nb))
        auto = gtime(lambda: C_.conv_fwd(x, w, s, s, p, p, True, sums=sums))
        best = min(fwd, key=fwd.get)
        row["fwd"] = {"auto_us": round(auto, 2), "best": list(best), "best_us": round(fwd[best], 2),
                      "all": {",".join(map(str, k)): round(v, 2) for k, v in fwd.items()}}
        plans.append({"op": "fwd", "M": N * P * P, "K": K, "C": C, "R": R, "S": R, "stride": s, "pad": p,
                      "bm": best[0], "bn": best[1], "splits": best[2], "stages": best[3],
                      "us": round(fwd[best], 2), "auto_us": round(auto, 2)})
        # ---- data gradient with the producer's BN-backward epilogue (mode 1: BN + ReLU)
        if K % 64 == 0 and (s == 1 or R > 1):
            dy = torch.randn(N, K, P, P, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            yc = torch.randn_like(x)
            mean = torch.zeros(C, device="cuda")
            invstd = torch.ones(C, device="cuda")
            bsums = torch.zeros(_native.STAT_SLOTS * 2 * C, device="cuda", dtype=torch.float64)
            geo = dict(stride=2, H=H, W=H) if s == 2 else {}
            nkd = R * R * K // 64

            wgk = dict(wg_x=x, wg_R=R, wg_S=R, wg_sh=s, wg_sw=s, wg_ph=p, wg_pw=p)
            dfn = C_.conv_dgrad_wgrad if a.dual else C_.conv_dgrad

            def dg(bm=-1, bn=-1, sp=-1, nb=0):
                kw = dict(wgk) if a.dual else {}
                return dfn(dy, w, p, p, bm, bn, sp, bn_x=yc, bn_mean=mean, bn_invstd=invstd, bn_mode=1,
                           bn_sums=bsums, stages=nb, **geo, **kw)

            dgr = {}
            for cfg in configs(nkd, strided_dgrad=s == 2 or a.dual):
                bm, bn, sp, nb = cfg
                dgr[cfg] = gtime(lambda: dg(bm, bn, sp, nb))
            auto = gtime(lambda: dg())
            best = min(dgr, key=dgr.get)
            row["dgrad_bnb"] = {"auto_us": round(auto, 2), "best": list(best), "best_us": round(dgr[best], 2),
                                "all": {",".join(map(str, k)): round(v, 2) for k, v in dgr.items()}}
            if a.dual:  # the fused launch's own knobs at that plan: weight-gradient split-K, grid order
                bm0, bn0, sp0, nb0 = best
                dual = {}
                for wsp in (-1, 2, 4, 8, 16, 32):
                    for order in (0, 1):
                        try:
                            dual[(wsp, order)] = gtime(lambda: C_.conv_dgrad_wgrad(
                                dy, w, p, p, bm0, bn0, sp0, bn_x=yc, bn_mean=mean, bn_invstd=invstd, bn_mode=1,
                                bn_sums=bsums, stages=nb0, order=order, **geo, **dict(wgk, wg_splits=wsp)))
                        except RuntimeError:
                            pass
                if dual:
                    bd = min(dual, key=dual.get)
                    row["dual_knobs"] = {"best": list(bd), "best_us": round(dual[bd], 2),
                                         "all": {",".join(map(str, k)): round(v, 2) for k, v in dual.items()}}
                    plans.append({"op": "wgrad_dual", "M": N * P * P, "K": K, "C": C, "R": R, "S": R, "stride": s,
                                  "pad": p, "bm": 64, "bn": 64, "splits": bd[0], "stages": 0, "order": bd[1],
                                  "us": round(dual[bd], 2), "auto_us": round(dual.get((-1, 1), dual[bd]), 2)})
            plans.append({"op": "dgrad_bnb", "M": N * H * H, "K": C, "C": K, "R": R, "S": R, "stride": s, "pad": p,
                          "bm": best[0], "bn": best[1], "splits": best[2], "stages": best[3],
                          "us": round(dgr[best], 2), "auto_us": round(auto, 2)})
            # the full-register variant: producer BN + residual + ReLU (mode 2: y read) with the
            # shortcut-gradient addend (a block's first conv) — its own plan key ("dgrad_bnb2")
            yy = torch.relu(torch.randn_like(x))
            add = torch.randn_like(x)

            def dg2(bm=-1, bn=-1, sp=-1, nb=0):
                kw = dict(wgk) if a.dual else {}
                return dfn(dy, w, p, p, bm, bn, sp, addend=add, bn_x=yc, bn_y=yy, bn_mean=mean,
                           bn_invstd=invstd, bn_mode=2, bn_sums=bsums, stages=nb, **geo, **kw)

            dg2r = {}
            for cfg in configs(nkd, strided_dgrad=s == 2 or a.dual):
                bm, bn, sp, nb = cfg
                dg2r[cfg] = gtime(lambda: dg2(bm, bn, sp, nb))
            auto = gtime(lambda: dg2())
            best = min(dg2r, key=dg2r.get)
            row["dgrad_bnb2"] = {"auto_us": round(auto, 2), "best": list(best), "best_us": round(dg2r[best], 2)}
            plans.append({"op": "dgrad_bnb2", "M": N * H * H, "K": C, "C": K, "R": R, "S": R, "stride": s, "pad": p,
                          "bm": best[0], "bn": best[1], "splits": best[2], "stages": best[3],
                          "us": round(dg2r[best], 2), "auto_us": round(auto, 2)})
        # ---- plain data gradient (block-input convs: no BN epilogue); 1x1 stride-2 runs on the output grid
        if K % 64 == 0 and (s == 1 or R > 1 or (R == 1 and p == 0)):
            s1x1 = R == 1 and s == 2
            dy = torch.randn(N, K, P, P, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            geo = dict(stride=2, H=H, W=H) if (s == 2 and R > 1) else {}
            nkd = R * R * K // 64
            pd = {}
            wgp = dict(wg_x=x, wg_R=R, wg_S=R, wg_sh=s, wg_sw=s, wg_ph=p, wg_pw=p) if a.dual else {}
            dfp = C_.conv_dgrad_wgrad if a.dual else C_.conv_dgrad
            for cfg in configs(nkd, strided_dgrad=(s == 2 and R > 1) or a.dual):
                bm, bn, sp, nb = cfg
                pd[cfg] = gtime(lambda: dfp(dy, w, p, p, bm, bn, sp, stages=nb, **geo, **wgp))
            auto = gtime(lambda: dfp(dy, w, p, p, **geo, **wgp))
            best = min(pd, key=pd.get)
            row["dgrad"] = {"auto_us": round(auto, 2), "best": list(best), "best_us": round(pd[best], 2)}
            Mg = N * P * P if s1x1 else N * H * H
            plans.append({"op": "dgrad", "M": Mg, "K": C, "C": K, "R": R, "S": R, "stride": 1 if s1x1 else s,
                          "pad": p, "bm": best[0], "bn": best[1], "splits": best[2], "stages": best[3],
                          "us": round(pd[best], 2), "auto_us": round(auto, 2)})
        # ---- weight gradient: tiles x pixel splits (the deferred reduce is off while timing)
        if C % 64 == 0 and K % 8 == 0:
            dy = torch.randn(N, K, P, P, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            wg = {}
            for bm in (64, 128):
                for bn in (64, 128):
                    if C % bn or (bm == 128 and K < 128):
                        continue
                    for sp in (-1, 8, 16, 32, 64, 96, 128):
                        try:
                            wg[(bm, bn, sp, 0)] = gtime(lambda: C_.conv_wgrad(dy, x, R, R, s, s, p, p, bm, bn, sp))
                        except RuntimeError:
                            pass
            auto = gtime(lambda: C_.conv_wgrad(dy, x, R, R, s, s, p, p))
            best = min(wg, key=wg.get)
            row["wgrad"] = {"auto_us": round(auto, 2), "best": list(best), "best_us": round(wg[best], 2)}
            if wg[best] < auto:
                plans.append({"op": "wgrad", "M": N * P * P, "K": K, "C": C, "R": R, "S": R, "stride": s, "pad": p,
                              "bm": best[0], "bn": best[1], "splits": best[2], "stages": 0,
                              "us": round(wg[best], 2), "auto_us": round(auto, 2)})
        raw.append(row)
        print(json.dumps({k: v for k, v in row.items() if k not in ("fwd", "dgrad_bnb", "dgrad_bnb2", "dgrad", "wgrad",
                                                                     "dual_knobs")}),
              json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "all"} for k, v in row.items()
                          if k in ("fwd", "dgrad_bnb", "dgrad_bnb2", "dgrad", "wgrad", "dual_knobs")}), flush=True)
    doc = {"device": torch.cuda.get_device_name(), "batch": a.batch,
           "note": "native conv launch plans by GEMM shape (M = output pixels, K = output channels, C = "
                   "reduction channels); written by scripts/conv_tune.py",
           "plans": plans}
    for path, obj in ((a.out, doc), (a.raw, raw)):
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as f:
            json.dump(obj, f, indent=1)
    for op in ("fwd", "dgrad_bnb", "dgrad_bnb2", "dgrad", "wgrad", "wgrad_dual"):
        ps = [pl for pl in plans if pl["op"] == op]
        print(json.dumps({"op": op, "n": len(ps), "sum_auto_us": round(sum(pl["auto_us"] for pl in ps), 1),
                          "sum_best_us": round(sum(pl["us"] for pl in ps), 1)}))


if __name__ == "__main__":
    main()
