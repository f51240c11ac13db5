#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/conv_timeline.py --out gpurun_out/r04/conv_timeline.json > gpurun_out/r04/conv_timeline.log 2>&1
echo rc=$?
cat gpurun_out/r04/conv_timeline.log | tail -8
