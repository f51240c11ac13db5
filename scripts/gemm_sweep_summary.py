"""One line per shape from scripts/gemm_pp_sweep.py output: vendor vs the best native (tile, splits).
    python scripts/gemm_sweep_summary.py sweep.jsonl"""
import json
import sys

for line in open(sys.argv[1]):
    r = json.loads(line)
    print(f"{r['layout']} {r['M']:>5} {r['N']:>5} {r['K']:>5}  vendor {r['vendor_us']:7.1f} us ({r['vendor_tf']:5.0f} TF)  "
          f"native {r['best']:>6} {r['best_us']:7.1f} us ({r['best_tf']:5.0f} TF)  native/vendor speed x{r['native_over_vendor']:.2f}")
