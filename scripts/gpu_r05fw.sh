#!/bin/bash
# round 5: one-wave attention forward grid for few (b, h) pairs — numerics + Llama A/B (interleaved)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05fw; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn_ln.py tests/test_gpu_llama_fused.py tests/test_gpu_llm_ops.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for nw in 0 1; do
    HYPERION_ATTN_FWD_NARROW=$nw timeout -k 10 400 python scripts/run_model_step.py llamagraph20 > $O/llama_${nw}_$i.log 2>&1 || { tail -5 $O/llama_${nw}_$i.log; exit 1; }
    echo "narrow=$nw run $i $(grep '^{' $O/llama_${nw}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
