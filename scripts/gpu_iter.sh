#!/bin/bash
# Fast GPU iteration: one test file (or -k filter), then bench (graph + eager) and a kernel-trace profile.
# Usage: bash scripts/gpu_iter.sh "<pytest args>" [prof]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "[iter] $(date +%T) $n"; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "[iter] $n rc=$rc"; tail -n 6 gpurun_out/$n.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest_iter 300 python3 -u -m pytest $1 -x -q -rf --timeout 120 --timeout-method thread
run bench_graph 300 python3 bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench_graph.json
run bench_eager 300 python3 bench.py --steps 30 --warmup 10 --graph 0 --json-out gpurun_out/bench_eager.json
if [ "${2:-}" = prof ]; then
  run prof_bench 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_bench" -o run -- python3 "$PWD/bench.py" --steps 10 --warmup 5 --graph 0
fi
echo "[iter] done"
