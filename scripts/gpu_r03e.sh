#!/bin/bash
# Round 3 re-entry evidence: smoke, headline bench, full GPU suite, Llama fused graphed step,
# FSDP world-1 steps (eager vs segmented graph), trainer fast paths
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 300 python3 __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log | cut -c1-200; fatal $rc
timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-220; fatal $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20; tail -3 gpurun_out/pytest_gpu.log; fatal $rc
timeout -k 10 300 python3 -u scripts/run_model_step.py llamagraph20 > gpurun_out/llama_fused.json 2> gpurun_out/llama_fused.err; rc=$?; echo "llama fused rc=$rc"; tail -1 gpurun_out/llama_fused.json | cut -c1-300; fatal $rc
for m in lm256 gpt2_small llama7b_lora; do
  for g in "" graph; do
    timeout -k 10 300 python3 -u scripts/run_model_step.py fsdp $m $g > gpurun_out/fsdp_${m}_${g:-eager}.json 2> gpurun_out/fsdp_${m}_${g:-eager}.err; rc=$?; echo "fsdp $m $g rc=$rc"; tail -1 gpurun_out/fsdp_${m}_${g:-eager}.json | cut -c1-300; fatal $rc
  done
done
timeout -k 10 300 python3 -u scripts/run_model_step.py fsdp llama7b_lora graph shardbase > gpurun_out/fsdp_llama_shardbase.json 2> gpurun_out/fsdp_llama_shardbase.err; rc=$?; echo "fsdp llama shardbase rc=$rc"; tail -1 gpurun_out/fsdp_llama_shardbase.json | cut -c1-300; fatal $rc
