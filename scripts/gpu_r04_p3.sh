#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-p3}
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/r04/bench_$tag.json 2> gpurun_out/r04/bench_$tag.err
echo bench rc=$?; cut -c1-160 gpurun_out/r04/bench_$tag.json
timeout -k 10 300 python -u scripts/ce_bench.py --out gpurun_out/r04/ce_bench_$tag.json > gpurun_out/r04/ce_bench_$tag.log 2>&1
echo ce rc=$?; grep -v amdgpu.ids gpurun_out/r04/ce_bench_$tag.log | cut -c1-900
timeout -k 10 300 python -u scripts/dbg_fsdp_coll.py > gpurun_out/r04/dbg_fsdp_$tag.log 2>&1
echo dbg rc=$?; grep -E "^coll|Error|error" gpurun_out/r04/dbg_fsdp_$tag.log | cut -c1-300
