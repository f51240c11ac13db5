#!/bin/bash
# FSDP segmented-capture tests + world-1 FSDP steps (eager vs graph), then kernel traces of the
# ResNet-50 bench step and the Llama-2-7B LoRA graphed step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fsdp_graph.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_fsdpg.log 2>&1; rc=$?; echo "fsdp graph tests rc=$rc"; grep -E "FAILED|Error" gpurun_out/pytest_fsdpg.log | head; tail -1 gpurun_out/pytest_fsdpg.log; fatal $rc
for m in lm256 gpt2_small llama7b_lora; do
  for g in "" graph; do
    timeout -k 10 300 python3 -u scripts/run_model_step.py fsdp $m $g > gpurun_out/fsdp_${m}_${g:-eager}.json 2> gpurun_out/fsdp_${m}_${g:-eager}.err; rc=$?; echo "fsdp $m $g rc=$rc"; tail -1 gpurun_out/fsdp_${m}_${g:-eager}.json | cut -c1-300; fatal $rc
  done
done
timeout -k 10 300 python3 -u scripts/run_model_step.py fsdp llama7b_lora graph shardbase > gpurun_out/fsdp_llama_shardbase.json 2> gpurun_out/fsdp_llama_shardbase.err; rc=$?; echo "fsdp llama shardbase rc=$rc"; tail -1 gpurun_out/fsdp_llama_shardbase.json | cut -c1-300; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/trace_bench" -o run -- python3 "$PWD/bench.py" --steps 6 --warmup 4 > gpurun_out/trace_bench.log 2>&1; rc=$?; echo "trace bench rc=$rc"; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/trace_llama" -o run -- python3 "$PWD/scripts/run_model_step.py" llamagraph > gpurun_out/trace_llama.log 2>&1; rc=$?; echo "trace llama rc=$rc"
