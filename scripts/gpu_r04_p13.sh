#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-p13}
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -q --timeout 450 --timeout-method thread tests/test_gpu_round4.py tests/test_gpu_debug_build.py > gpurun_out/r04/pytest_$tag.log 2>&1
rc=$?; echo tests rc=$rc; tail -2 gpurun_out/r04/pytest_$tag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/r04/bench_$tag.json 2> gpurun_out/r04/bench_$tag.err
echo bench rc=$?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04/bench_$tag.json | head -1
bash scripts/gpu_r04_trace.sh trace_$tag > /dev/null 2>&1; echo trace rc=$?; grep -E "step -2" gpurun_out/r04/trace_$tag/step.txt
