#!/bin/bash
# Round-4 iteration loop: ResNet-50 bench + native conv per-shape timings (no vendor baselines).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
tag=${1:-quick}
shift || true
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/r04/bench_$tag.json 2> gpurun_out/r04/bench_$tag.err && \
timeout -k 10 300 python -u scripts/conv_roofline.py --vendor 0 "$@" --out gpurun_out/r04/conv_$tag.json > gpurun_out/r04/conv_$tag.log 2>&1 && \
cat gpurun_out/r04/bench_$tag.json && tail -1 gpurun_out/r04/conv_$tag.log
