#!/bin/bash
# round 5, call Q: where the 2-rank gloo segmented bench step spends its host time
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05q; mkdir -p $O
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
HYPERION_SEG_PROFILE=1 HYPERION_DIST_BACKEND=gloo HYPERION_COMM=torch timeout -k 10 300 $TR --nproc-per-node 2 --master-port 29661 bench.py --gpus 2 --steps 3 --warmup 2 > $O/seg.log 2>&1 || { tail -30 $O/seg.log; exit 1; }
grep '^{' $O/seg.log | python -c "import json,sys; r=json.loads(sys.stdin.readline()); print(r['ms_per_step'], r['config']['ddp_schedule']); print(r.get('seg_host_profile'))"
HYPERION_SEG_PROFILE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ddp-world1 1 > $O/seg1.log 2>&1 || { tail -30 $O/seg1.log; exit 1; }
grep '^{' $O/seg1.log | python -c "import json,sys; r=json.loads(sys.stdin.readline()); print(r['ms_per_step'], r['config']['ddp_schedule']); print(r.get('seg_host_profile'))"
