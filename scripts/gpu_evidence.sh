#!/bin/bash
# Evidence run: baseline rows (fp32 reference methodology + bf16 Hyperion), ResNet-50 batch sweep,
# FSDP steps (LM-256 / GPT-2-small / Llama-2-7B LoRA, world 1), fused-vs-eager inference.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/models
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for part in ${*:-fsdp fusion baseline scaling}; do
  echo "[ev] $(date +%T) $part"
  timeout -k 10 400 python3 -u -m hyperion.cli.bench_models --only $part --out gpurun_out/models/$part > gpurun_out/models/$part.log 2>&1
  rc=$?; echo "[ev] $part rc=$rc"; tail -n 6 gpurun_out/models/$part.log | cut -c1-400
  [ $rc -ne 0 ] && exit $rc
done
echo done
