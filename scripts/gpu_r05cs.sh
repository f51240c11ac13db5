#!/bin/bash
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05cs; mkdir -p $O
timeout -k 10 300 python scripts/micro/copy_sources.py vit > $O/vit.txt 2>&1 || { tail -20 $O/vit.txt; exit 1; }
timeout -k 10 300 python scripts/micro/copy_sources.py gpt2 > $O/gpt2.txt 2>&1 || { tail -20 $O/gpt2.txt; exit 1; }
grep -v "amdgpu.ids\|Warning\|warn" $O/vit.txt | head -30
echo ----
grep -v "amdgpu.ids\|Warning\|warn" $O/gpt2.txt | head -30
