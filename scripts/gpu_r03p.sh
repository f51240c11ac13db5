#!/bin/bash
# FSDP world-1 steps: eager vs segmented-graph, Llama with the frozen base sharded (replicate_frozen=False)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fsdp_r03
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for args in "lm256 graph" "gpt2_small graph" "llama7b_lora graph" "llama7b_lora graph shardbase" "llama7b_lora shardbase"; do
  timeout -k 10 240 python3 -u scripts/run_model_step.py fsdp $args > gpurun_out/fsdp_r03/run.log 2>&1; rc=$?
  grep '^{' gpurun_out/fsdp_r03/run.log | tail -1 >> gpurun_out/fsdp_r03/fsdp_steps.jsonl
  echo "$args rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/fsdp_r03/run.log; exit $rc; }
done
exit 0
