#!/bin/bash
# Round-2 re-entry evidence: headline bench, full GPU suite, kernel traces of the ResNet-50 and
# Llama-2-7B LoRA graphed steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench_graph.json > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; fatal $rc
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/trace_bench" -o run -- python3 "$PWD/bench.py" --steps 6 --warmup 4 > gpurun_out/trace_bench.log 2>&1; rc=$?; echo "trace rc=$rc"; fatal $rc
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/trace_llama" -o run -- python3 "$PWD/scripts/run_model_step.py" llamagraph > gpurun_out/trace_llama.log 2>&1; rc=$?; echo "llama trace rc=$rc"; grep "^{" gpurun_out/trace_llama.log | cut -c1-200; fatal $rc
echo done
