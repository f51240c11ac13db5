#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_fsdp_graph.py tests/test_gpu_ddp_segments.py tests/test_gpu_ddp_graph.py > gpurun_out/r04/pytest_dp_p8.log 2>&1
echo dp rc=$?; tail -2 gpurun_out/r04/pytest_dp_p8.log


