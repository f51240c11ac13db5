"""Per-workgroup timeline of one conv_fwd launch (diagnostic stamps, csrc/kernels/conv_igemm.hip):
entry / before K loop / after K loop / end in s_memrealtime ticks (100 MHz) plus HW_ID / XCC_ID, and
inside the epilogue: after the LDS transpose and after the store loop (8 words per workgroup).

Prints, per configuration, the kernel span, the per-workgroup phase medians (prologue, K loop,
epilogue), how many workgroups ran concurrently per CU, and how long a K step takes.  The stamp's
own fences slow the kernel a little: read the shares, not the absolute span.

    python scripts/conv_timeline.py [--out gpurun_out/conv_timeline.json]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402

CASES = [  # op, N, C, H, K, R, stride, pad, bm, bn, splits
    ("fwd", 32, 256, 14, 256, 3, 1, 1, -1, -1, -1),
    ("fwd", 32, 64, 56, 256, 1, 1, 0, -1, -1, -1),
    ("dgrad", 32, 256, 56, 64, 1, 1, 0, -1, -1, -1),
    ("dgrad_bnb", 32, 256, 56, 64, 1, 1, 0, -1, -1, -1),
    ("dgrad", 32, 256, 56, 128, 1, 1, 0, -1, -1, -1),
    ("dgrad_bnb", 32, 256, 56, 128, 1, 1, 0, -1, -1, -1),
    ("dgrad_bnb", 32, 256, 56, 128, 1, 1, 0, 64, 64, 1),
    ("dgrad", 32, 512, 28, 128, 1, 1, 0, -1, -1, -1),
    ("dgrad_bnb", 32, 512, 28, 128, 1, 1, 0, -1, -1, -1),
    ("dgrad_bnb", 32, 64, 56, 64, 3, 1, 1, -1, -1, -1),
]


def analyse(st):
    st = st[st[:, 0] != 0]
    t0 = int(st[:, 0].min())
    s = (st[:, :4] - t0).double() * 10.0 / 1000.0  # us
    hw, xcc = st[:, 4], st[:, 5]
    # CU key: XCC_ID, then HW_ID's se_id [15:13], sh_id [12], cu_id [11:8]
    cu = (xcc & 0xF) * 4096 + ((hw >> 13) & 0x7) * 64 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 0xF)
    pro = (s[:, 1] - s[:, 0]).tolist()
    loop = (s[:, 2] - s[:, 1]).tolist()
    epi = (s[:, 3] - s[:, 2]).tolist()
    sd = (st[:, 6:8] - t0).double() * 10.0 / 1000.0
    has = st[:, 6] != 0
    transp = (sd[has, 0] - s[has, 2]).tolist()
    stores = (sd[has, 1] - sd[has, 0]).tolist()
    tail = (s[has, 3] - sd[has, 1]).tolist()
    tot = (s[:, 3] - s[:, 0]).tolist()
    # concurrency per CU: max overlapping [start, end) intervals among workgroups on one CU
    per_cu = {}
    for i in range(st.shape[0]):
        per_cu.setdefault(int(cu[i]), []).append((float(s[i, 0]), float(s[i, 3])))
    conc = []
    for iv in per_cu.values():
        ev = sorted([(a, 1) for a, _ in iv] + [(b, -1) for _, b in iv])
        c = m = 0
        for _, d in ev:
            c += d
            m = max(m, c)
        conc.append(m)
    starts = sorted(s[:, 0].tolist())
    med = statistics.median
    return {
        "wgs": int(st.shape[0]), "cus_used": len(per_cu), "span_us": round(float(s[:, 3].max()), 2),
        "prologue_us_med": round(med(pro), 2), "loop_us_med": round(med(loop), 2), "epilogue_us_med": round(med(epi), 2),
        "epi_transpose_us_med": round(med(transp), 2) if transp else None,
        "epi_stores_us_med": round(med(stores), 2) if stores else None,
        "epi_tail_us_med": round(med(tail), 2) if tail else None,
        "wg_total_us_med": round(med(tot), 2), "wg_total_us_max": round(max(tot), 2),
        "max_concurrent_per_cu": max(conc), "median_concurrent_per_cu": med(conc),
        "last_start_us": round(starts[-1], 2), "start_p50_us": round(starts[len(starts) // 2], 2),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/conv_timeline.json")
    a = ap.parse_args()
    C_ = _native.native()
    rows = []
    buf = torch.zeros(200000 * 8, dtype=torch.int64, device="cuda")
    for (op, N, C, H, K, R, s, p, bm, bn, sp) in CASES:
        x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, C, R, R, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
        P0 = (H + 2 * p - R) // s + 1
        dy = torch.randn(N, K, P0, P0, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        mean, invstd = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        bs = torch.zeros(_native.STAT_SLOTS * 2 * C, device="cuda", dtype=torch.float64)

        def run():
            if op == "fwd":
                return C_.conv_fwd(x, w, s, s, p, p, True, bm, bn, sp)
            if op == "dgrad":
                return C_.conv_dgrad(dy, w, p, p, bm, bn, sp)
            return C_.conv_dgrad(dy, w, p, p, bm, bn, sp, bn_x=x, bn_mean=mean, bn_invstd=invstd, bn_mode=1,
                                 bn_sums=bs)

        for _ in range(5):
            run()
        torch.cuda.synchronize()
        buf.zero_()
        C_.conv_set_stamps(buf)
        run()
        torch.cuda.synchronize()
        C_.conv_set_stamps(None)
        st = buf.view(-1, 8).cpu()
        nk = R * R * C // 64
        P = (H + 2 * p - R) // s + 1
        r = dict(op=op, N=N, C=C, H=H, K=K, R=R, stride=s, pad=p, bm=bm, bn=bn, splits=sp, nk=nk, M=N * P * P)
        r.update(analyse(st))
        rows.append(r)
        print(json.dumps(r), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
