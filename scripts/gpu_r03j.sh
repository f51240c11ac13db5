#!/bin/bash
# LoRA kernels: numerics + PMC counters per kernel (two passes) over scripts/lora_bench.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_llama_fused.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lora.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_lora.log; grep -E "^E .*(assert|Error)" gpurun_out/pytest_lora.log | head -5
[ $rc -le 1 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d "$PWD/gpurun_out/pmc_lora1" -o run -- python3 "$PWD/scripts/lora_bench.py" > gpurun_out/pmc_lora1.log 2>&1; echo "pmc1 rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$PWD/gpurun_out/pmc_lora2" -o run -- python3 "$PWD/scripts/lora_bench.py" > gpurun_out/pmc_lora2.log 2>&1; echo "pmc2 rc=$?"
timeout -k 10 100 python3 -u scripts/lora_bench.py 2>/dev/null
