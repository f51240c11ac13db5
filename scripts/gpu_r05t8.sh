#!/bin/bash
# round 5: 4-wave 256x128 GEMM tile (tile 8) — numerics, sweep vs tile 1 / vendor, model steps
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05t8; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_tiled.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
GEMM_TN="768 3072 6304,3072 768 6304,2304 768 6304,768 768 6304,768 3072 2048,2304 768 2048" timeout -k 10 400 python scripts/micro/gemm_sweep.py 6304 3072 768 6304 768 3072 2048 3072 768 8192 8192 8192 > $O/sweep.jsonl 2>&1 || { tail -5 $O/sweep.jsonl; exit 1; }
grep -v amdgpu $O/sweep.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    if 'tn' in d: print(d['tn'], 'vendor', d['vendor'], 'best', d['best'], d[d['best']], d['best_tf'], 't1best', min([v for k,v in d.items() if k.startswith('t1s')], default=None), 't8best', min([v for k,v in d.items() if k.startswith('t8s')], default=None))
    else: print(d['M'],d['N'],d['K'], 'vendor', d['vendor']['warm_us'], 't1', d.get('t1',{}).get('warm_us') if isinstance(d.get('t1'),dict) else d.get('t1'), 't8', d['t8']['warm_us'] if isinstance(d.get('t8'),dict) else d.get('t8'))
"
for m in vitgraph gpt2; do
  timeout -k 10 300 python scripts/run_model_step.py $m > $O/$m.log 2>&1 || { tail -5 $O/$m.log; exit 1; }
  echo "$m $(grep '^{' $O/$m.log | grep -o '"ms_per_step": [0-9.]*')"
  grep '^{' $O/$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('gemm_choices'))"
done
