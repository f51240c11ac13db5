#!/bin/bash
# conv plan tuning (fwd / dgrad_bnb / dgrad / wgrad), then the bench with the fresh plans vs the kept ones.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-p9}
mkdir -p gpurun_out/r04
timeout -k 10 1000 python -u scripts/conv_tune.py --out gpurun_out/r04/conv_plans_$tag.json --raw gpurun_out/r04/conv_tune_raw_$tag.json > gpurun_out/r04/conv_tune_$tag.log 2>&1
echo tune rc=$?; tail -4 gpurun_out/r04/conv_tune_$tag.log
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/r04/bench_${tag}_kept.json 2>/dev/null && \
HYPERION_CONV_PLANS=$PWD/gpurun_out/r04/conv_plans_$tag.json timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/r04/bench_${tag}_new.json 2>/dev/null
echo bench rc=$?; cut -c1-140 gpurun_out/r04/bench_${tag}_kept.json gpurun_out/r04/bench_${tag}_new.json
