#!/bin/bash
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05dbg; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_debug_build.py -q --timeout 500 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; exit $rc
