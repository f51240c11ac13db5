#!/bin/bash
# round 5, call J: batched DDP bucket packs (copy_mt) + zero-arena stage fallback — DDP tests,
# world-1 DDP schedule A/B, a trace of the segmented schedule
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05j; mkdir -p $O
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] rc=$rc"; grep -E "passed|failed|^\{" $O/$n.log | cut -c1-330 | tail -3; [ $rc -eq 0 ] || { tail -25 $O/$n.log; exit $rc; }; }
step pytest 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ddp_graph.py tests/test_gpu_ddp_segments.py tests/test_gpu_round4.py
for sched in auto segmented; do
  for cd in fp32 bf16; do
    step ddp1_${sched}_${cd} 200 python bench.py --steps 50 --warmup 10 --ddp-world1 1 --ddp-schedule $sched --comm-dtype $cd
  done
done
step bench_default 150 python bench.py --steps 50 --warmup 10
bash scripts/gpu_r05_trace.sh ddp_seg_j --ddp-world1 1 --ddp-schedule segmented || exit 1
