#!/bin/bash
# A/B: loss kernel and fc path on the ResNet-50 bench (3 runs each, alternating)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04/ab
for i in 1 2; do
  for v in base fused; do
    case $v in
      base) env_=""; arg="";;
      fused) env_=""; arg="--loss fused";;
      fcnat) env_="HYPERION_RESNET_FC=native"; arg="";;
    esac
    env $env_ timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 $arg > gpurun_out/r04/ab/$v.$i.json 2>/dev/null || exit 1
    echo $v $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04/ab/$v.$i.json | head -1)
  done
done
