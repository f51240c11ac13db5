#!/bin/bash
# round 5: attention query-split cap 2 vs 4 (auto) on the Llama LoRA step, interleaved
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05qs3; mkdir -p $O
for i in 1 2; do
  for qs in 2 0; do
    HYPERION_ATTN_QSPLIT=$qs timeout -k 10 400 python scripts/run_model_step.py llamagraph20 > $O/llama_${qs}_$i.log 2>&1 || { tail -5 $O/llama_${qs}_$i.log; exit 1; }
    echo "qsplit_cap=$qs run $i $(grep '^{' $O/llama_${qs}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
