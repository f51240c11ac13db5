#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-p7}
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_round4.py tests/test_gpu_llm_ops.py > gpurun_out/r04/pytest_$tag.log 2>&1
rc=$?; echo tests rc=$rc; tail -2 gpurun_out/r04/pytest_$tag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/r04/bench_$tag.json 2> gpurun_out/r04/bench_$tag.err
echo bench rc=$?; cut -c1-160 gpurun_out/r04/bench_$tag.json
timeout -k 10 300 python -u scripts/run_model_step.py gpt2 > gpurun_out/r04/gpt2_$tag.json 2>gpurun_out/r04/gpt2_$tag.err && \
timeout -k 10 300 python -u scripts/run_model_step.py vitgraph > gpurun_out/r04/vit_$tag.json 2>gpurun_out/r04/vit_$tag.err
echo models rc=$?; cut -c1-200 gpurun_out/r04/gpt2_$tag.json gpurun_out/r04/vit_$tag.json
timeout -k 10 300 python -u scripts/dbg_fsdp_coll.py > gpurun_out/r04/dbg_fsdp_$tag.log 2>&1
echo dbg rc=$?; grep -E "^coll|Error|error" gpurun_out/r04/dbg_fsdp_$tag.log | cut -c1-300
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_llama_full_fsdp.py > gpurun_out/r04/pytest_llamafull_$tag.log 2>&1
echo llamafull test rc=$?; tail -2 gpurun_out/r04/pytest_llamafull_$tag.log
for cfg in "lm256 graph" "gpt2_small graph" "llama7b_full curve"; do
  timeout -k 10 400 python -u scripts/run_model_step.py fsdp $cfg >> gpurun_out/r04/fsdp_steps_$tag.jsonl 2>>gpurun_out/r04/fsdp_steps_$tag.err || break
done
cut -c1-400 gpurun_out/r04/fsdp_steps_$tag.jsonl
