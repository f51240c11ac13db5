"""Per-kernel timeline of ONE training step from a rocprofv3 --kernel-trace CSV.

    python scripts/step_trace.py <run_kernel_trace.csv> [--step -2] [--out file]

Steps are delimited by the fused optimizer kernel (adam_mt_k ends every step).  Prints each kernel of
the chosen step in launch order (index, short name, grid, us) and a per-family summary.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    return n[:80]


ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--step", type=int, default=-2)
ap.add_argument("--out", default=None)
a = ap.parse_args()
rows = []
with open(a.csv) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                     r.get("Grid_Size", r.get("Grid_Size_X", "")), r.get("Workgroup_Size", "")))
rows.sort()
ends = [i for i, r in enumerate(rows) if "adam_mt_k" in r[2]]
bounds = [0] + [e + 1 for e in ends]
steps = [rows[bounds[i]:bounds[i + 1]] for i in range(len(bounds) - 1)]
st = steps[a.step]
lines = []
fam = defaultdict(lambda: [0, 0.0])
t0 = st[0][0]
for i, (s, e, n, g, w) in enumerate(st):
    us = (e - s) / 1e3
    lines.append(f"{i:4d} {(s - t0) / 1e3:9.1f} {us:8.1f}  grid={g:>8s} wg={w:>4s}  {n}")
    fam[n][0] += 1
    fam[n][1] += us
busy = sum((e - s) for s, e, *_ in st) / 1e3
span = (st[-1][1] - st[0][0]) / 1e3
lines.append(f"\nstep {a.step}: {len(st)} kernels, busy {busy:.1f} us, span {span:.1f} us")
for n, (c, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
    lines.append(f"{t:9.1f} us {c:4d}x  {n}")
txt = "\n".join(lines)
print(txt)
if a.out:
    open(a.out, "w").write(txt + "\n")
