#!/bin/bash
# round 5: attention query split A/B on the Llama LoRA step (interleaved), GPT-2 / LM-256 unchanged
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05qs2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn_ln.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for qs in 1 0; do
    HYPERION_ATTN_QSPLIT=$qs timeout -k 10 400 python scripts/run_model_step.py llamagraph20 > $O/llama_${qs}_$i.log 2>&1 || { tail -5 $O/llama_${qs}_$i.log; exit 1; }
    echo "qsplit=$qs run $i $(grep '^{' $O/llama_${qs}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
timeout -k 10 300 python scripts/run_model_step.py gpt2 > $O/gpt2.log 2>&1 && echo "gpt2 $(grep '^{' $O/gpt2.log | grep -o '"ms_per_step": [0-9.]*')"
