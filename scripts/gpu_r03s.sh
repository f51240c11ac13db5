#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fsdp_r03c
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn_ln.py tests/test_gpu_fsdp_graph.py tests/test_gpu_llama_fused.py tests/test_gpu_graph_step.py > gpurun_out/r03s_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03s_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/r03s_tests.log | head -20; exit $rc; }
: > gpurun_out/fsdp_r03c/fsdp_steps.jsonl
for args in "lm256 graph" "gpt2_small graph" "llama7b_lora graph" "llama7b_lora graph shardbase"; do
  timeout -k 10 240 python3 -u scripts/run_model_step.py fsdp $args > gpurun_out/fsdp_r03c/run.log 2>&1; rc=$?
  grep '^{' gpurun_out/fsdp_r03c/run.log | tail -1 >> gpurun_out/fsdp_r03c/fsdp_steps.jsonl
  echo "$args rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/fsdp_r03c/run.log; exit $rc; }
done
exit 0
