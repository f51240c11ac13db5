"""A/B of the fp32 reference-methodology rows (bench/baseline.py, three timed loops): native fp32
convolutions (ops/conv_f32.py) vs the vendor kernels, same process, interleaved."""
import json
import sys

sys.path.insert(0, ".")
from hyperion.bench.baseline import baseline_suite, benchmark_model  # noqa: E402
from hyperion.ops import conv_f32  # noqa: E402

only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
for name, fn, ishape, tshape in baseline_suite(real_vit=True):
    if only and name not in only:
        continue
    for rep in range(2):
        for native in (False, True):
            conv_f32.ENABLED = native
            r = benchmark_model(fn, ishape, tshape, 20, 5, "fp32", "hyperion", name=name)
            r["conv_f32"] = native
            r["rep"] = rep
            print(json.dumps(r), flush=True)
