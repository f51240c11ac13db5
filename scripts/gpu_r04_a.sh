#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/stem_bench.py > gpurun_out/r04/stem_bench.json 2>gpurun_out/r04/stem_bench.err && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_round4.py > gpurun_out/r04/pytest_r4.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -v --timeout 500 --timeout-method thread tests/test_gpu_ddp_segments.py tests/test_gpu_ddp_graph.py > gpurun_out/r04/pytest_ddpg.log 2>&1
echo rc=$?
cat gpurun_out/r04/stem_bench.json; tail -3 gpurun_out/r04/pytest_r4.log; tail -4 gpurun_out/r04/pytest_ddpg.log
