#!/bin/bash
# forward / dgrad tile x ring-depth sweep over every ResNet-50 conv shape
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04/sweep
export TMPDIR=/tmp
for st in 1 2; do for t in 128,128,1 128,64,1 64,64,1 64,64,2; do
  timeout -k 10 200 python -u scripts/conv_roofline.py --vendor 0 --only fwd,dgrad --stages $st --tiles $t --out gpurun_out/r04/sweep/s${st}_${t//,/_}.json > gpurun_out/r04/sweep/s${st}_${t//,/_}.log 2>&1 || exit 1
done; done
echo done
