#!/bin/bash
# round 5, call P: the N>1 bench path rehearsed on one GPU — bench.py under torch.distributed.run
# with 2 ranks (gloo collectives between the processes, both on the one card), the segmented
# default and the 3-graph split; plus the single-rank native-RCCL launcher path (N=1 via torchrun)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05p; mkdir -p $O
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] rc=$rc"; grep -E "^\{" $O/$n.log | cut -c1-600 | tail -2; [ $rc -eq 0 ] || { tail -30 $O/$n.log; exit $rc; }; }
run tr1 300 $TR --nproc-per-node 1 --master-port 29651 bench.py --gpus 1 --steps 20 --warmup 5
HYPERION_DIST_BACKEND=gloo HYPERION_COMM=torch run gloo2_seg 400 $TR --nproc-per-node 2 --master-port 29652 bench.py --gpus 2 --steps 10 --warmup 3
HYPERION_DIST_BACKEND=gloo HYPERION_COMM=torch run gloo2_auto 400 $TR --nproc-per-node 2 --master-port 29653 bench.py --gpus 2 --steps 10 --warmup 3 --ddp-schedule auto
