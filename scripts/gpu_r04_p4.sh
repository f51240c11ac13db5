#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-p4}
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u scripts/dbg_fsdp_coll.py > gpurun_out/r04/dbg_fsdp_$tag.log 2>&1
echo dbg rc=$?; grep -E "^coll|Error|error" gpurun_out/r04/dbg_fsdp_$tag.log | cut -c1-400
