#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-p4}
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_llm_ops.py > gpurun_out/r04/pytest_llm_$tag.log 2>&1
rc=$?; echo llm tests rc=$rc; tail -3 gpurun_out/r04/pytest_llm_$tag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/dbg_fsdp_coll.py > gpurun_out/r04/dbg_fsdp_$tag.log 2>&1
echo dbg rc=$?; grep -E "^coll|Error|error" gpurun_out/r04/dbg_fsdp_$tag.log | cut -c1-400
timeout -k 10 300 python -u scripts/run_model_step.py lmgraph > gpurun_out/r04/lm256_$tag.json 2>gpurun_out/r04/lm256_$tag.err && \
timeout -k 10 300 python -u scripts/run_model_step.py gpt2 > gpurun_out/r04/gpt2_$tag.json 2>gpurun_out/r04/gpt2_$tag.err
echo lm rc=$?; cut -c1-250 gpurun_out/r04/lm256_$tag.json gpurun_out/r04/gpt2_$tag.json
python3 - <<PY
import json
for f in ("lm256", "gpt2"):
    try:
        r = json.load(open(f"gpurun_out/r04/{f}_$tag.json"))
        print(f, {k: v for k, v in r.get("gemm_choices", {}).items()})
    except Exception as e:
        print(f, e)
PY
