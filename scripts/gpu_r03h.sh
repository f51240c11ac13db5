#!/bin/bash
# LoRA kernels v3 (split-K lora_down with last-arriver sum, register-blocked lora_bwd_t / lora_bwd_a)
# + FSDP persistent first-gather fix: numerics, Llama step + trace, FSDP capture tests + steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_llama_fused.py tests/test_gpu_wstream.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lora.log 2>&1; rc=$?; echo "lora tests rc=$rc"; grep -E "FAILED|Error" gpurun_out/pytest_lora.log | head; tail -1 gpurun_out/pytest_lora.log; fatal $rc
timeout -k 10 300 python3 -u scripts/run_model_step.py llamagraph20 > gpurun_out/llama_fused.json 2> gpurun_out/llama_fused.err; rc=$?; echo "llama fused rc=$rc"; tail -1 gpurun_out/llama_fused.json | cut -c1-300; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/trace_llama" -o run -- python3 "$PWD/scripts/run_model_step.py" llamagraph > gpurun_out/trace_llama.log 2>&1; rc=$?; echo "trace llama rc=$rc"; fatal $rc
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fsdp_graph.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_fsdpg.log 2>&1; rc=$?; echo "fsdp graph tests rc=$rc"; grep -E "FAILED|Error" gpurun_out/pytest_fsdpg.log | head; tail -1 gpurun_out/pytest_fsdpg.log; fatal $rc
for m in lm256 gpt2_small llama7b_lora; do
  for g in "" graph; do
    timeout -k 10 300 python3 -u scripts/run_model_step.py fsdp $m $g > gpurun_out/fsdp_${m}_${g:-eager}.json 2> gpurun_out/fsdp_${m}_${g:-eager}.err; rc=$?; echo "fsdp $m $g rc=$rc"; tail -1 gpurun_out/fsdp_${m}_${g:-eager}.json | cut -c1-300; fatal $rc
  done
done
