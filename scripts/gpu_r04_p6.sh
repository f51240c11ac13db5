#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/gpu_r04_p5.sh p5 || exit $?
TUNE=1 bash scripts/gpu_r04_a.sh p6
