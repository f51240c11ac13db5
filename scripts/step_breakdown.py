"""Per-step kernel breakdown of a rocprofv3 kernel trace of bench.py (a group of adam_mt_k launches marks a step end).

Usage: python scripts/step_breakdown.py <run_kernel_trace.csv> [n_steps] [top]
"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    depth, out = 0, []
    for ch in name:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)[:120]


def main(path, n=5, top=40):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam_mt_k" in r["Kernel_Name"]]
    ends = [i for j, i in enumerate(adam) if j + 1 == len(adam) or adam[j + 1] > i + 16]  # one group per step
    a, b = ends[-n - 1], ends[-1]
    w = rows[a + 1:b + 1]
    span = (int(w[-1]["End_Timestamp"]) - int(w[0]["Start_Timestamp"])) / n / 1e3
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in w) / n / 1e3
    print(f"{n} steps: span {span:.0f} us/step, busy {busy:.0f} us/step, {len(w) / n:.0f} kernels/step")
    agg = collections.defaultdict(lambda: [0.0, 0.0])
    for r in w:
        k = short(r["Kernel_Name"])
        agg[k][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / n / 1e3
        agg[k][1] += 1 / n
    for k, v in sorted(agg.items(), key=lambda x: -x[1][0])[:top]:
        print(f"{v[0]:8.1f} us {v[1]:6.1f}x  {k}")


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:]))
