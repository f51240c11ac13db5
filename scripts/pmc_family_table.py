"""Per-kernel-family MFMA busy / LDS activity from one rocprofv3 --pmc counter CSV
(SQ_VALU_MFMA_BUSY_CYCLES, SQ_LDS_IDX_ACTIVE, SQ_LDS_BANK_CONFLICT, SQ_WAIT_INST_LDS, SQ_WAVE_CYCLES,
GRBM_GUI_ACTIVE): python scripts/pmc_family_table.py counter_collection.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    fam = name.split("(")[0].replace("void ", "")
    if "ws_gemm_k" in fam:
        fam = "hyp::ws_gemm_k<" + ("NN" if ", true," in name.split(">")[0] else "NT") + ">"
    fam = fam[:70]
    agg[fam][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[fam].add(r.get("Dispatch_Id"))
print("| kernel family | dispatches | MFMA busy % | LDS-active cycles per CU-cycle | bank-conflict / LDS cycle | LDS-wait share of wave time |")
print("|---|---|---|---|---|---|")
for fam, c in sorted(agg.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0))[:12]:
    g = c.get("GRBM_GUI_ACTIVE", 0) / 8.0  # summed over the 8 XCDs -> cycles
    if g <= 0:
        continue
    mfma = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (g * 1024)
    lds, conf = c.get("SQ_LDS_IDX_ACTIVE", 0), c.get("SQ_LDS_BANK_CONFLICT", 0)
    wl = c.get("SQ_WAIT_INST_LDS", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1)
    print(f"| `{fam}` | {len(disp[fam])} | {mfma:.1f} | {lds / (g * 256):.2f} | {conf / max(lds - conf, 1):.2f} | {wl:.3f} |")
