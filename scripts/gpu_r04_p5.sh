#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-p5}
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u scripts/dbg_fsdp_coll.py > gpurun_out/r04/dbg_fsdp_$tag.log 2>&1
echo dbg rc=$?; grep -E "^coll|Error|error" gpurun_out/r04/dbg_fsdp_$tag.log | cut -c1-300
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_fsdp_graph.py tests/test_gpu_ddp_segments.py tests/test_gpu_ddp_graph.py > gpurun_out/r04/pytest_dp_$tag.log 2>&1
echo dp tests rc=$?; tail -3 gpurun_out/r04/pytest_dp_$tag.log
timeout -k 10 300 python -u scripts/gemm_probe.py --out gpurun_out/r04/gemm_probe_$tag.json > gpurun_out/r04/gemm_probe_$tag.log 2>&1
echo probe rc=$?; python3 - <<PY
import json
for r in json.load(open("gpurun_out/r04/gemm_probe_$tag.json")):
    print(r["shape"], "ven", r["vendor_us"], "ven_gemm", r["vendor_gemm_only_us"], "nat", r["native_best"], "plan", r["plan"])
PY
