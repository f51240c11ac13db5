#!/bin/bash
# round 5: GEMM autotune vendor-side timing without the stray add (ViT / GPT-2 graphed steps)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05z2; mkdir -p $O
for i in 1 2; do
  for m in vitgraph gpt2 vitckptgraph; do
    timeout -k 10 300 python scripts/run_model_step.py $m > $O/${m}_$i.log 2>&1 || { tail -5 $O/${m}_$i.log; exit 1; }
    echo "$m $i $(grep '^{' $O/${m}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
grep '^{' $O/vitgraph_1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('gemm_choices'))"
