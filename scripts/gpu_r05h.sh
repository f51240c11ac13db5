#!/bin/bash
# round 5, call H: segmented DDP schedule + non-blocking optimizer tables — tests, DDP schedule A/B,
# ViT-B/16 + checkpointing graphed, fp32/bf16 model benchmark rows
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05h; mkdir -p $O
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] rc=$rc"; grep -E "passed|failed|^\{" $O/$n.log | cut -c1-400 | tail -4; [ $rc -eq 0 ] || { tail -25 $O/$n.log; exit $rc; }; }
step pytest 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ddp_graph.py tests/test_gpu_bn_adam.py tests/test_gpu_graph_step.py
step bench_default 150 python bench.py --steps 50 --warmup 10
step ddp1_auto 200 python bench.py --steps 50 --warmup 10 --ddp-world1 1
step ddp1_seg 200 python bench.py --steps 50 --warmup 10 --ddp-world1 1 --ddp-schedule segmented
step ddp1_auto_bf16 200 python bench.py --steps 50 --warmup 10 --ddp-world1 1 --comm-dtype bf16
step ddp1_seg_bf16 200 python bench.py --steps 50 --warmup 10 --ddp-world1 1 --ddp-schedule segmented --comm-dtype bf16
step ddp1_seg_b25 200 python bench.py --steps 50 --warmup 10 --ddp-world1 1 --ddp-schedule segmented --bucket-mb 25
step vitckptgraph 300 python scripts/run_model_step.py vitckptgraph
step vitgraph 300 python scripts/run_model_step.py vitgraph
step models 900 python -u -m hyperion.cli.bench_models --only baseline --out $O/models
