#!/bin/bash
# final evidence: FSDP world-1 steps (graph / eager / sharded base), reference-API trainer steps, model benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
: > gpurun_out/final/fsdp_steps.jsonl
for args in "lm256 graph" "gpt2_small graph" "llama7b_lora graph" "llama7b_lora graph shardbase" "lm256" "gpt2_small"; do
  timeout -k 10 240 python3 -u scripts/run_model_step.py fsdp $args > gpurun_out/final/run.log 2>&1; rc=$?
  grep '^{' gpurun_out/final/run.log | tail -1 >> gpurun_out/final/fsdp_steps.jsonl
  echo "fsdp $args rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/final/run.log; exit $rc; }
done
timeout -k 10 600 python3 -u scripts/trainer_steps.py > gpurun_out/final/trainer_steps.jsonl 2> gpurun_out/final/trainer_steps.err; rc=$?; echo "trainers rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u -m hyperion.cli.bench_models --only lm,llama --out gpurun_out/final/models > gpurun_out/final/models.log 2>&1; rc=$?; echo "models rc=$rc"
exit $rc
