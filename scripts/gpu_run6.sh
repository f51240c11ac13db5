#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "[run] $(date +%T) $n"; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "[run] $n rc=$rc"; tail -n 4 gpurun_out/$n.log | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest_conv 300 python3 -m pytest tests/test_gpu_conv.py -q -x
run pytest_gpu 600 python3 -m pytest tests -m gpu -q --deselect tests/test_gpu_comm.py
run bench_graph 300 python3 bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench_graph.json
run bench_eager 300 python3 bench.py --steps 30 --warmup 10 --graph 0 --json-out gpurun_out/bench_eager.json
run prof_eager 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_eager2" -o run -- python3 "$PWD/bench.py" --steps 10 --warmup 3 --graph 0
run models 900 python3 -m hyperion.cli.bench_models --out gpurun_out/models --only lm,vit,llama,fusion

run pytest_comm 200 python3 -X faulthandler -m pytest tests/test_gpu_comm.py -q -x
echo "[run] done"
