#!/bin/bash
# round 5, call R: DDP world-1 schedules — segmented with native RCCL vs torch no-op comm, ONE graph
# with the RCCL all-reduces captured; tests of the one-graph schedule
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05r; mkdir -p $O
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] rc=$rc"; grep -E "passed|failed" $O/$n.log | tail -2; grep '^{' $O/$n.log | python -c "import json,sys; r=json.loads(sys.stdin.readline()); print(r['ms_per_step'], r['host_ms_per_step'], r['config']['ddp_schedule'], r['final_loss'])" 2>/dev/null; [ $rc -eq 0 ] || { tail -25 $O/$n.log; exit $rc; }; }
step pytest 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ddp_graph.py
step plain 150 python bench.py --steps 50 --warmup 10
step seg_native 200 python bench.py --steps 50 --warmup 10 --ddp-world1 1
HYPERION_COMM=torch step seg_torch 200 python bench.py --steps 50 --warmup 10 --ddp-world1 1
step graph_native 200 python bench.py --steps 50 --warmup 10 --ddp-world1 1 --ddp-schedule graph
step graph_native_bf16 200 python bench.py --steps 50 --warmup 10 --ddp-world1 1 --ddp-schedule graph --comm-dtype bf16
step seg_native_b256 200 python bench.py --steps 50 --warmup 10 --ddp-world1 1 --bucket-mb 256
