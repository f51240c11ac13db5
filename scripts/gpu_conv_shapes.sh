#!/bin/bash
# Conv kernel numerics, then per-layer ResNet-50 conv timings (fwd / dgrad / wgrad, ours vs MIOpen,
# LDS pipeline-depth sweep).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_conv.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -c "
import json, sys; sys.path.insert(0, '.')
from hyperion.bench.conv_shapes import run
rows = run(32, sweep=True)
json.dump(rows, open('gpurun_out/conv_shapes.json', 'w'), indent=1)
" > gpurun_out/conv_shapes.log 2>&1
rc=$?; echo "shapes rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench_graph.json > gpurun_out/bench_graph.log 2>&1
echo "bench rc=$?"; tail -1 gpurun_out/bench_graph.log | cut -c1-200
