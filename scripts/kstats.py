"""Top kernels of a rocprofv3 kernel trace CSV: python scripts/kstats.py trace.csv [n] [skip_first_fraction]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
skip = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[int(len(rows) * skip):]
k = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k[r["Kernel_Name"][:150]][0] += 1
    k[r["Kernel_Name"][:150]][1] += d
tot = sum(v[1] for v in k.values())
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"kernels {len(rows)}  busy {tot/1e3:.2f} ms  span {span/1e3:.2f} ms")
for name, (c, t) in sorted(k.items(), key=lambda x: -x[1][1])[:n]:
    print(f"{t/1e3:8.2f} ms {100*t/tot:5.1f}% {c:6d}  {t/c:8.1f} us  {name}")
