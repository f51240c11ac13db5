#!/bin/bash
# round 5: LayerNorm grid sweep (HYPERION_LN_WAVES) on the ViT / GPT-2 graphed steps
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05ln; mkdir -p $O
for w in 0 3200 6400 1024; do
  for m in vitgraph gpt2; do
    HYPERION_LN_WAVES=$w timeout -k 10 300 python scripts/run_model_step.py $m > $O/${m}_$w.log 2>&1 || { tail -5 $O/${m}_$w.log; exit 1; }
    echo "waves=$w $m $(grep '^{' $O/${m}_$w.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
HYPERION_LN_WAVES=6400 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn_ln.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
