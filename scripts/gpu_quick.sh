#!/bin/bash
# Quick GPU iteration: selected GPU tests, then the 1-GPU bench (graph) and a kernel-trace profile.
# Usage: bash scripts/gpu_quick.sh "<pytest -k expr or test files>" [prof]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "[q] $(date +%T) $n"; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "[q] $n rc=$rc"; tail -n 4 gpurun_out/$n.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
TESTS=${1:-tests}
run pytest_q 400 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread
run bench_q 300 python3 bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench_q.json
if [ "${2:-}" = prof ]; then
  run prof_q 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_q" -o run -- python3 "$PWD/bench.py" --steps 10 --warmup 5 --graph 0
  python3 scripts/step_breakdown.py gpurun_out/prof_q/run_kernel_trace.csv 5 30
fi
