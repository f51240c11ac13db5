#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-p10}
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_round4.py tests/test_gpu_conv.py > gpurun_out/r04/pytest_$tag.log 2>&1
rc=$?; echo tests rc=$rc; tail -2 gpurun_out/r04/pytest_$tag.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_p9.sh $tag
