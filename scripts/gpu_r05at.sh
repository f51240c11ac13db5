#!/bin/bash
# round 5: attention skips fully padded query / key blocks (S = 197) — numerics + ViT / GPT-2 steps
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05at; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn_ln.py tests/test_gpu_llm_ops.py tests/test_gpu_dropout_graphs.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/attn_bench.py > $O/attn_bench.log 2>&1 || { tail -10 $O/attn_bench.log; exit 1; }
grep -v amdgpu $O/attn_bench.log | tail -12
for m in vitgraph gpt2 vitgraph; do
  timeout -k 10 300 python scripts/run_model_step.py $m > $O/$m.log 2>&1 || { tail -5 $O/$m.log; exit 1; }
  echo "$m $(grep '^{' $O/$m.log | grep -o '"ms_per_step": [0-9.]*')"
done
