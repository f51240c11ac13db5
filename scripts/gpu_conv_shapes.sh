#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python3 -c "
import json, sys; sys.path.insert(0, '.')
from hyperion.bench.conv_shapes import run
rows = run(32)
json.dump(rows, open('gpurun_out/conv_shapes.json', 'w'), indent=1)
" > gpurun_out/conv_shapes.log 2>&1
echo rc=$?
timeout -k 10 900 python3 -m hyperion.cli.bench_models --out gpurun_out/models --only lm,llama > gpurun_out/models2.log 2>&1
echo rc=$?
