#!/bin/bash
# LM / GPT-2 steps with bf16 compute copies, FSDP steps (grouped grad landing, deferred clip)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fsdp_r03b gpurun_out/models
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fsdp_graph.py tests/test_gpu_bn_adam.py tests/test_gpu_graph_step.py > gpurun_out/r03r_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03r_tests.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/r03r_tests.log; exit $rc; }
timeout -k 10 400 python3 -u -m hyperion.cli.bench_models --only lm --out gpurun_out/models/lm_r03b > gpurun_out/models/lm_r03b.log 2>&1; rc=$?; echo "lm rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/models/lm_r03b.log; exit $rc; }
: > gpurun_out/fsdp_r03b/fsdp_steps.jsonl
for args in "lm256 graph" "gpt2_small graph" "llama7b_lora graph" "llama7b_lora graph shardbase" "gpt2_small"; do
  timeout -k 10 240 python3 -u scripts/run_model_step.py fsdp $args > gpurun_out/fsdp_r03b/run.log 2>&1; rc=$?
  grep '^{' gpurun_out/fsdp_r03b/run.log | tail -1 >> gpurun_out/fsdp_r03b/fsdp_steps.jsonl
  echo "$args rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/fsdp_r03b/run.log; exit $rc; }
done
exit 0
