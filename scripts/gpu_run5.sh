#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "[run] $(date +%T) $n"; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "[run] $n rc=$rc"; tail -n 4 gpurun_out/$n.log | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest_gpu 600 python3 -m pytest tests -m gpu -q
run bench_graph 300 python3 bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench_graph.json
run models 900 python3 -m hyperion.cli.bench_models --out gpurun_out/models --only lm,vit,llama,fusion
run baseline 900 python3 -m hyperion.cli.bench_models --out gpurun_out/models --only baseline
echo "[run] done"
