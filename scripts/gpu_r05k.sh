#!/bin/bash
# round 5, call K: 2-rank segmented DDP test, host time per step of the bench schedules,
# CustomTransformer eager host profile (fp32 / bf16 / torch) + kernel stats
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05k; mkdir -p $O
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] rc=$rc"; grep -E "passed|failed|^\{" $O/$n.log | cut -c1-200 | tail -3; [ $rc -eq 0 ] || { tail -25 $O/$n.log; exit $rc; }; }
step pytest 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ddp_graph.py -k "two_rank or segmented"
step bench_default 150 python bench.py --steps 50 --warmup 10
step ddp1_seg 200 python bench.py --steps 50 --warmup 10 --ddp-world1 1
python -c "
import json
for n in ['bench_default','ddp1_seg']:
    for l in open('$O/'+n+'.log'):
        if l.startswith('{'): r=json.loads(l); print(n, r['ms_per_step'], 'host', r['host_ms_per_step'])
"
step ct32 200 python scripts/eager_host_prof.py ct32
step ct16 200 python scripts/eager_host_prof.py ct16
HYPERION_KERNELS=torch step ct32_torch 200 python scripts/eager_host_prof.py ct32
for v in ct32 ct16; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_$v" -o run -- python3 "$PWD/scripts/eager_host_prof.py" $v > $O/prof_$v.log 2>&1 || exit 1
done
HYPERION_KERNELS=torch timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_ct32_torch" -o run -- python3 "$PWD/scripts/eager_host_prof.py" ct32 > $O/prof_ct32_torch.log 2>&1 || exit 1
find $O -name "*kernel_trace.csv" -delete
echo ok
