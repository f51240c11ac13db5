#!/bin/bash
# round-3 checkpoint: full GPU suite, smoke, headline bench + kernel trace, ViT-B/16 graphed traces
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head -20; tail -2 gpurun_out/pytest_gpu.log; fatal $rc
timeout -k 10 300 python3 __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log | cut -c1-200; fatal $rc
timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-220; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/trace_bench" -o run -- python3 "$PWD/bench.py" --steps 6 --warmup 4 > gpurun_out/trace_bench.log 2>&1; rc=$?; echo "trace bench rc=$rc"; fatal $rc
bash scripts/gpu_vit_trace.sh
timeout -k 10 300 python3 -u scripts/run_model_step.py llamagraph20 > gpurun_out/llama_fused.json 2> gpurun_out/llama_fused.err; rc=$?; echo "llama fused rc=$rc"; tail -1 gpurun_out/llama_fused.json | cut -c1-200; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/trace_llama" -o run -- python3 "$PWD/scripts/run_model_step.py" llamagraph > gpurun_out/trace_llama.log 2>&1; echo "trace llama rc=$?"
