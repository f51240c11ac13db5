"""Per-kernel-family summary of the LAST complete training step in a rocprofv3 kernel trace (steps end
at the optimizer kernel).  python scripts/step_summary.py <run_kernel_trace.csv> [top]"""
import collections
import csv
import re
import sys


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)[:100]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
ends = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
# a step with several Adam launches (bf16 compute copies + fp32 masters): keep the last of each run
ends = [i for j, i in enumerate(ends) if j + 1 == len(ends) or ends[j + 1] != i + 1]
st = rows[ends[-2] + 1:ends[-1] + 1] if len(ends) > 1 else rows
agg = collections.defaultdict(lambda: [0, 0.0])
for r in st:
    k = short(r["Kernel_Name"])
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
busy = sum(v[1] for v in agg.values())
span = (int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"])) / 1e3
print(f"one step: {len(st)} kernels, busy {busy:.0f} us, span {span:.0f} us")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{v[1]:9.1f} us {v[0]:5d}x  {k}")
