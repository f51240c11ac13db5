#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gpu_round4.py -k "strided_conv_bn" > gpurun_out/r04/pytest_r4b.log 2>&1
echo rc=$?
timeout -k 10 200 python -u scripts/conv_timeline.py --out gpurun_out/r04/conv_timeline2.json > gpurun_out/r04/conv_timeline2.log 2>&1
echo rc=$?
tail -3 gpurun_out/r04/pytest_r4b.log; cut -c1-520 gpurun_out/r04/conv_timeline2.log
