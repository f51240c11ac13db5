"""Per-kernel-family table from the llama_pmc.sh passes: time share, bytes/s, TLB and L2 behaviour.
    python scripts/ws_pmc_table.py gpurun_out/r06/llama_pmc"""
import csv
import re
import sys
from collections import defaultdict

d = sys.argv[1]


def fam(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    m = re.match(r"([\w:]+?)(<|\(|$)", name)
    base = m.group(1) if m else name[:40]
    if "ws_gemm_k" in name:  # NT vs NN instances
        base += "<NN>" if re.search(r"ws_gemm_k<[^,]+, \d+, \d+, true", name) else "<NT>"
    return base[:60]


agg = defaultdict(lambda: defaultdict(float))
for i in range(1, 6):
    try:
        rows = list(csv.DictReader(open(f"{d}/llama_P{i}.csv")))
    except FileNotFoundError:
        continue
    seen = defaultdict(set)
    for r in rows:
        k = fam(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        seen[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    for k, s in seen.items():
        agg[k][f"disp{i}"] = len(s)
dur = defaultdict(float)
try:
    for r in csv.DictReader(open(f"{d}/kernel_trace.csv")):
        dur[fam(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
except FileNotFoundError:
    pass
tot = sum(dur.values()) or 1.0
print("| kernel family | trace s (share) | EA rd GB/s | DRAM rd GB/s | UTCL1 miss % | multi-miss stalls | L2 hit % | rd latency cyc | wait % |")
print("|---|---|---|---|---|---|---|---|---|")
for k in sorted(dur, key=lambda k: -dur[k])[:14]:
    a = agg.get(k, {})
    t = dur[k]
    n = a.get("disp2", 1) or 1
    ea = a.get("TCC_EA0_RDREQ_sum", 0) * 64 / t / 1e9 if t else 0  # EA read requests of 64 B (approx.)
    dram = a.get("TCC_EA0_RDREQ_DRAM_sum", 0) * 64 / t / 1e9 if t else 0
    mh = a.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0) + a.get("TCP_UTCL1_TRANSLATION_HIT_sum", 0)
    miss = 100 * a.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0) / mh if mh else float("nan")
    l2 = a.get("TCC_HIT_sum", 0) + a.get("TCC_MISS_sum", 0)
    hit = 100 * a.get("TCC_HIT_sum", 0) / l2 if l2 else float("nan")
    lat = a.get("TCP_TCC_READ_REQ_LATENCY_sum", 0) / a["TCP_TCC_READ_REQ_sum"] if a.get("TCP_TCC_READ_REQ_sum") else float("nan")
    wait = 100 * a.get("SQ_WAIT_ANY", 0) / a["SQ_WAVE_CYCLES"] if a.get("SQ_WAVE_CYCLES") else float("nan")
    print(f"| {k} | {t:.4f} ({100 * t / tot:.1f}%) | {ea:.0f} | {dram:.0f} | {miss:.1f} | "
          f"{a.get('TCP_UTCL1_STALL_MULTI_MISS_sum', 0):.3g} | {hit:.1f} | {lat:.0f} | {wait:.1f} |")
