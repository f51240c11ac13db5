#!/bin/bash
# round 5, call L: split-K reduce in the last-arriving workgroup — GEMM / linear tests, probe A/B,
# GPT-2 and ViT graphed steps A/B
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05l; mkdir -p $O
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] rc=$rc"; grep -E "passed|failed|^\{" $O/$n.log | cut -c1-300 | tail -3; [ $rc -eq 0 ] || { tail -25 $O/$n.log; exit $rc; }; }
step pytest 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_tiled.py tests/test_gpu_linear.py tests/test_gpu_gemm.py
step probe_inkernel 400 python scripts/gemm_probe.py --out $O/probe_inkernel.json
HYPERION_SPLITK_INKERNEL=0 step probe_separate 400 python scripts/gemm_probe.py --out $O/probe_separate.json
python - <<PY
import json
a=json.load(open('$O/probe_inkernel.json')); b=json.load(open('$O/probe_separate.json'))
for x,y in zip(a,b):
    ks=[k for k in x if k.startswith('t') and '_s' in k and not k.endswith('s1') and not k.endswith('s-1')]
    print(x['shape'], 'best in', x['native_best'], 'sep', y['native_best'], 'vendor', x['vendor_us'], x['vendor_gemm_only_us'], {k:(x[k], y.get(k)) for k in ks if k.startswith('t2')})
PY
step gpt2_in 300 python scripts/run_model_step.py gpt2
HYPERION_SPLITK_INKERNEL=0 step gpt2_sep 300 python scripts/run_model_step.py gpt2
step vit_in 300 python scripts/run_model_step.py vitgraph
HYPERION_SPLITK_INKERNEL=0 step vit_sep 300 python scripts/run_model_step.py vitgraph
