#!/bin/bash
# round 5: attention backward query split for S <= 128 (Llama 32 heads at batch 1) — numerics + A/B
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05qs; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn_ln.py tests/test_gpu_llama_fused.py tests/test_gpu_llm_ops.py tests/test_gpu_dropout_graphs.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for qs in 1 0; do
  for m in llamagraph gpt2 lmgraph; do
    HYPERION_ATTN_QSPLIT=$qs timeout -k 10 400 python scripts/run_model_step.py $m > $O/${m}_$qs.log 2>&1 || { tail -5 $O/${m}_$qs.log; exit 1; }
    echo "qsplit=$qs $m $(grep '^{' $O/${m}_$qs.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
