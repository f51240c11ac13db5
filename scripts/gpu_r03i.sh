#!/bin/bash
# LoRA kernel micro-timings, launch floor under env knobs, FSDP capture tests + steps (frozen groups
# resident at world 1), weight-streaming plan sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 120 python3 -u scripts/lora_bench.py > gpurun_out/lora_bench.json 2> gpurun_out/lora_bench.err; rc=$?; echo "lora bench rc=$rc"; tail -1 gpurun_out/lora_bench.json; fatal $rc
timeout -k 10 120 python3 -u scripts/launch_floor2.py default > gpurun_out/floor_default.json 2>/dev/null; rc=$?; echo "floor rc=$rc"; cat gpurun_out/floor_default.json; fatal $rc
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 120 python3 -u scripts/launch_floor2.py pktcap1 > gpurun_out/floor_pkt1.json 2>/dev/null; echo "rc=$?"; cat gpurun_out/floor_pkt1.json
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python3 -u scripts/launch_floor2.py pktcap0 > gpurun_out/floor_pkt0.json 2>/dev/null; echo "rc=$?"; cat gpurun_out/floor_pkt0.json
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python3 -u scripts/launch_floor2.py devkernarg > gpurun_out/floor_kernarg.json 2>/dev/null; echo "rc=$?"; cat gpurun_out/floor_kernarg.json
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fsdp_graph.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_fsdpg.log 2>&1; rc=$?; echo "fsdp graph tests rc=$rc"; grep -E "FAILED|Error" gpurun_out/pytest_fsdpg.log | head; tail -1 gpurun_out/pytest_fsdpg.log; fatal $rc
for m in lm256 gpt2_small llama7b_lora; do
  for g in "" graph; do
    timeout -k 10 300 python3 -u scripts/run_model_step.py fsdp $m $g > gpurun_out/fsdp_${m}_${g:-eager}.json 2> gpurun_out/fsdp_${m}_${g:-eager}.err; rc=$?; echo "fsdp $m $g rc=$rc"; tail -1 gpurun_out/fsdp_${m}_${g:-eager}.json | cut -c1-360; fatal $rc
  done
done
timeout -k 10 400 python3 -u scripts/ws_bench.py > gpurun_out/ws_bench.log 2>&1; rc=$?; echo "ws bench rc=$rc"; grep -v amdgpu gpurun_out/ws_bench.log | cut -c1-600
