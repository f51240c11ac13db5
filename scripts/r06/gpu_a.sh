#!/bin/bash
# round-6 GPU batch A: GEMM + LM head + selective-recompute tests, GEMM sweep, model steps
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r06/a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_tiled.py \
  tests/test_gpu_llm_ops.py tests/test_gpu_gemm.py tests/test_gpu_linear.py > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/r06/gemm_pp_sweep.py --big > $O/sweep.jsonl 2> $O/sweep.err || { tail -5 $O/sweep.err; exit 1; }
python3 -c "
import json
for l in open('$O/sweep.jsonl'):
    r=json.loads(l); print(r['layout'],r['M'],r['N'],r['K'],'vendor',r['vendor_us'],'best',r['best'],r['best_us'],'x%.2f'%r['native_over_vendor'], 'pp', {k:v for k,v in r.items() if k[:3] in ('t8s','t9s','t10','t11','t12')})
"
for m in vitgraph vitselgraph vitckptgraph gpt2 lmgraph; do
  timeout -k 10 400 python -u scripts/run_model_step.py $m > $O/$m.json 2> $O/$m.err || { echo "[$m] FAILED"; tail -5 $O/$m.err; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/$m.json').read().strip().splitlines()[-1]); print('$m', round(r['ms_per_step'],3), 'ms peak', round(r.get('peak_mem_mb',0)), 'MB')"
done
