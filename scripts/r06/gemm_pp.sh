#!/bin/bash
# ping-pong GEMM tiles: numerics tests, then the native-vs-vendor sweep
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r06/gemm_pp; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_tiled.py tests/test_gpu_llm_ops.py tests/test_gpu_gemm.py tests/test_gpu_linear.py > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/r06/gemm_pp_sweep.py --big > $O/sweep.jsonl 2> $O/sweep.err || { tail -5 $O/sweep.err; exit 1; }
python3 -c "
import json
for l in open('$O/sweep.jsonl'):
    r=json.loads(l); print(r['layout'],r['M'],r['N'],r['K'],'vendor',r['vendor_us'],'best',r['best'],r['best_us'],'x%.2f'%r['native_over_vendor'], {k:v for k,v in r.items() if k.startswith('t8') or k.startswith('t9') or k.startswith('t10') or k.startswith('t11')})
"
