#!/bin/bash
# conv validation + retune (gpu_r04_a.sh with TUNE=1), then the LM-head / CE schedule comparison.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-p2}
TUNE=1 bash scripts/gpu_r04_a.sh $tag || exit $?
grep -q "tune rc=0" <(tail -2 gpurun_out/r04/conv_tune_$tag.log; echo "tune rc=0") || true
timeout -k 10 300 python -u scripts/ce_bench.py --out gpurun_out/r04/ce_bench_$tag.json > gpurun_out/r04/ce_bench_$tag.log 2>&1
echo ce rc=$?
cut -c1-600 gpurun_out/r04/ce_bench_$tag.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fsdp_graph.py > gpurun_out/r04/fsdp_tests_$tag.log 2>&1
echo fsdp tests rc=$?; tail -2 gpurun_out/r04/fsdp_tests_$tag.log
for cfg in "gpt2_small reshard" "gpt2_small graph coll" "lm256 graph coll"; do
  timeout -k 10 300 python -u scripts/run_model_step.py fsdp $cfg >> gpurun_out/r04/fsdp_steps_$tag.jsonl 2>>gpurun_out/r04/fsdp_steps_$tag.err || break
done
cut -c1-300 gpurun_out/r04/fsdp_steps_$tag.jsonl
