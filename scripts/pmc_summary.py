"""Summarize rocprofv3 --pmc passes into a per-kernel roofline table.

    python scripts/pmc_summary.py gpurun_out/pmc [--out profiles/pmc_r02.md]

Layout: <dir>/<target>_<PASS>/run_counter_collection.csv (one pass = one run).  Per kernel
(hyp:: kernels, plus torch's add for the STREAM A/B) the counters are averaged per dispatch and
combined across passes:
  MfmaUtil %  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)  (rocprof's
                definition; the per-dispatch CSV sums GRBM_GUI_ACTIVE over the 8 XCDs' GRBMs, rocprof's
                derived metric takes their max)
  MFMA TF/s   = SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 / kernel time
  HBM rd GB/s = 2 * FETCH_SIZE (KiB) / time   (gfx950 FETCH_SIZE counts half of 16-B-per-lane reads:
                MI355X_MICROARCH.md §HBM)
  HBM wr GB/s = WRITE_SIZE (KiB) / time
  L2 hit %    = TCC_HIT / (TCC_HIT + TCC_MISS)
  LDS conflict = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS  (extra cycles per LDS instruction)
  waves/CU    = SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs)  (mean resident waves per CU)
  wait %      = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES  (wave-cycles stalled waiting on any instruction)
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name[:90]


def load(path):
    per = defaultdict(lambda: defaultdict(float))  # kernel -> counter -> sum over dispatches
    disp = defaultdict(set)
    dur = defaultdict(dict)
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            if not (k.startswith("hyp::") or "CUDAFunctor_add" in k or "vectorized_elementwise" in k or "Cijk" in k):
                continue
            d = int(r["Dispatch_Id"])
            disp[k].add(d)
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[k][d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # us
    out = {}
    for k in per:
        n = len(disp[k])
        c = {name: v / n for name, v in per[k].items()}
        c["_n"] = n
        c["_us"] = sum(dur[k].values()) / n
        out[k] = c
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    merged = defaultdict(dict)  # (target, kernel) -> counters
    for d in sorted(glob.glob(os.path.join(a.dir, "*_*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.isfile(f):
            continue
        target = os.path.basename(d).rsplit("_", 1)[0]
        for k, c in load(f).items():
            m = merged[(target, k)]
            us = m.get("_us_list", [])
            us.append(c["_us"])
            m.update({kk: v for kk, v in c.items() if not kk.startswith("_")})
            m["_us_list"] = us
            m["_n"] = c["_n"]
    lines = ["| target | kernel | dispatches | us/dispatch | MfmaUtil % | MFMA TF/s | HBM rd GB/s | HBM wr GB/s | L2 hit % | LDS confl/inst | waves/CU | wait % | parked % |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for (t, k), c in sorted(merged.items()):
        us = min(c["_us_list"])  # the SQ pass perturbs timing least
        def g(name):
            return c.get(name)
        util = 100 * g("SQ_VALU_MFMA_BUSY_CYCLES") / (g("GRBM_GUI_ACTIVE") / 8 * 1024) if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE") else None
        tf = g("SQ_INSTS_VALU_MFMA_MOPS_BF16") * 512 / (us * 1e-6) / 1e12 if g("SQ_INSTS_VALU_MFMA_MOPS_BF16") else None
        rd = 2 * g("FETCH_SIZE") * 1024 / (us * 1e-6) / 1e9 if g("FETCH_SIZE") is not None else None
        wr = g("WRITE_SIZE") * 1024 / (us * 1e-6) / 1e9 if g("WRITE_SIZE") is not None else None
        hit = 100 * g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")) if g("TCC_HIT_sum") is not None and (g("TCC_HIT_sum") + g("TCC_MISS_sum")) > 0 else None
        lds = g("SQ_LDS_BANK_CONFLICT") / g("SQ_INSTS_LDS") if g("SQ_INSTS_LDS") else None
        occ = g("SQ_WAVE_CYCLES") / (g("GRBM_GUI_ACTIVE") / 8 * 256) if g("SQ_WAVE_CYCLES") and g("GRBM_GUI_ACTIVE") else None
        wait = 100 * g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES") if g("SQ_WAIT_INST_ANY") and g("SQ_WAVE_CYCLES") else None
        parked = 100 * g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES") if g("SQ_WAIT_ANY") and g("SQ_WAVE_CYCLES") else None
        f = lambda v, p=1: "-" if v is None else f"{v:.{p}f}"  # noqa: E731
        lines.append(f"| {t} | `{k}` | {c['_n']} | {us:.1f} | {f(util)} | {f(tf, 0)} | {f(rd, 0)} | {f(wr, 0)} | {f(hit)} | "
                     f"{f(lds, 2)} | {f(occ)} | {f(wait)} | {f(parked)} |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
