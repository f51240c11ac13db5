#!/bin/bash
# round 5, call N: grid-filling GEMM tiles (64x64, 128x64, 64x128, 192x128) — tests, probe, GPT-2 /
# ViT / LM graphed steps with the autotuner choosing among them
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05n; mkdir -p $O
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] rc=$rc"; grep -E "passed|failed|^\{" $O/$n.log | cut -c1-250 | tail -3; [ $rc -eq 0 ] || { tail -25 $O/$n.log; exit $rc; }; }
step pytest 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_tiled.py tests/test_gpu_linear.py tests/test_gpu_gemm.py
step probe 500 python scripts/gemm_probe.py --out $O/probe.json
python - <<PY
import json
for x in json.load(open('$O/probe.json')):
    print(x['shape'], 'best', x['native_best'], 'vendor', x['vendor_us'], x['vendor_gemm_only_us'], {k: x[k] for k in x if k[:2] in ('t4','t5','t6','t7') and k.endswith(('_s1','_s2','_s3'))})
PY
step gpt2 300 python scripts/run_model_step.py gpt2
step vit 300 python scripts/run_model_step.py vitgraph
step vitckpt 300 python scripts/run_model_step.py vitckptgraph
step lm 300 python scripts/run_model_step.py lmgraph
python - <<PY
import json
for n in ['gpt2','vit','vitckpt','lm']:
    for l in open('$O/'+n+'.log'):
        if l.startswith('{'):
            r=json.loads(l); ch=r.get('gemm_choices') or {}
            print(n, round(r['ms_per_step'],3), 'vendor shapes', sum(1 for v in ch.values() if v is None), 'of', len(ch), ch)
PY
