#!/bin/bash
# Reference entry points on one GPU (torchrun, 1 rank): every trainer for a few steps + RCCL check.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cli
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
TR="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611"
run() { local n=$1 t=$2; shift 2; echo "[$n] $(date +%T)"; timeout -k 10 $t "$@" > gpurun_out/cli/$n.log 2>&1; local rc=$?; echo "[$n] rc=$rc"; tail -n 3 gpurun_out/cli/$n.log | cut -c1-250; if [ $rc -ne 0 ]; then grep -v "^\s*$" gpurun_out/cli/$n.log | grep -B30 -m1 "Error\|error:" | head -60; exit $rc; fi; }
run language_ddp 300 $TR -m hyperion.cli.run_distributed --model language_ddp --epochs 2 --max_steps 20 --dataset_size 2048 --base_dir /tmp/hyp_run
run cifar 300 $TR -m hyperion.cli.run_distributed --model cifar --epochs 2 --max_steps 20 --dataset_size 2048 --base_dir /tmp/hyp_run
run language_fsdp 300 $TR -m hyperion.cli.run_distributed --model language_fsdp --epochs 2 --max_steps 20 --dataset_size 2048 --base_dir /tmp/hyp_run
run llama_lora 500 $TR -m hyperion.cli.run_distributed --model llama --lora --epochs 1 --max_steps 10 --dataset_size 64 --base_dir /tmp/hyp_run --no_save
run test_rccl 120 $TR -m hyperion.cli.test_rccl
ls /tmp/hyp_run/data/distributed 2>/dev/null | head
echo done
