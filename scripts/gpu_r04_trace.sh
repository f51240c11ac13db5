#!/bin/bash
# rocprofv3 kernel trace of the ResNet-50 bench step (+ per-step kernel table / timeline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-trace}
mkdir -p gpurun_out/r04/$tag
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r04/$tag/prof" -o run -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/r04/$tag/bench.json 2> gpurun_out/r04/$tag/bench.err && \
f=$(ls gpurun_out/r04/$tag/prof/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/r04/$tag/prof/run_kernel_trace.csv) && \
python3 scripts/step_trace.py $f --step -2 --out gpurun_out/r04/$tag/step.txt > /dev/null && \
python3 scripts/kstats.py $f > gpurun_out/r04/$tag/kstats.txt 2>&1
echo rc=$?
cat gpurun_out/r04/$tag/bench.json | cut -c1-200; head -40 gpurun_out/r04/$tag/kstats.txt
