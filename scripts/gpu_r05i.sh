#!/bin/bash
# round 5, call I: deep-ring GEMM tiles (tests + probe) and kernel traces of the two world-1 DDP schedules
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_tiled.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python scripts/gemm_probe.py --out $O/gemm_probe.json > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
python -c "
import json
for r in json.load(open('$O/gemm_probe.json')):
    print(r['shape'], 'best', r['native_best'], 'vendor', r['vendor_us'], r['vendor_gemm_only_us'], {k: v for k, v in r.items() if k[:2] in ('t4', 't5')})
"
bash scripts/gpu_r05_trace.sh ddp_auto --ddp-world1 1 || exit 1
bash scripts/gpu_r05_trace.sh ddp_seg --ddp-world1 1 --ddp-schedule segmented || exit 1
