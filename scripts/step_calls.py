"""List every kernel of the last bench step in a rocprofv3 kernel trace (duration, grid, regs).

Usage: python scripts/step_calls.py <run_kernel_trace.csv> [kernels_per_step] [name_filter]
"""
import csv
import re
import sys


def main(path, per_step=524, filt=""):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))[-per_step:]
    for r in rows:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        n = re.sub(r"\(.*", "", n)[:70]
        if filt and filt not in n:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        print(f"{d:7.2f} {wg:6d}x{r['Grid_Size_Y']:>4}x{r['Grid_Size_Z']:>3} lds{r['LDS_Block_Size']:>6} "
              f"v{r['VGPR_Count']:>4}/{r['Accum_VGPR_Count']:>3} {n}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 524, sys.argv[3] if len(sys.argv) > 3 else "")
