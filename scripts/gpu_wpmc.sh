#!/bin/bash
# PMC passes over single wgrad configs (scripts/wgrad_probe.py --one): one rocprofv3 run per pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wpmc
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for cfg in "$@"; do
  for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d "$PWD/gpurun_out/wpmc/p$i" -o run -- python3 scripts/wgrad_probe.py --one "$cfg" > gpurun_out/wpmc/p$i.log 2>&1
    rc=$?; echo "pass $i cfg=$cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/wpmc/kt" -o run -- python3 scripts/wgrad_probe.py --one "$1" > gpurun_out/wpmc/kt.log 2>&1; echo "kt rc=$?"
