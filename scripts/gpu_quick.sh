#!/bin/bash
# Quick GPU iteration: selected test files, ResNet-50 bench (graph + eager), Llama LoRA graph step.
# Usage: bash scripts/gpu_quick.sh "<test files>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "[$n] rc=$rc"; grep -E "passed|failed|^\{" gpurun_out/$n.log | cut -c1-260 | tail -3; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$n.log; exit $rc; fi; }
run pytest 300 python3 -u -m pytest $1 -x -q --timeout 120 --timeout-method thread
run bench_graph 300 python3 bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench_graph.json
run bench_eager 300 python3 bench.py --steps 30 --warmup 10 --graph 0 --json-out gpurun_out/bench_eager.json
run llamagraph 400 python3 scripts/run_model_step.py llamagraph
