#!/bin/bash
# round 5, call Z: conv tile-order group sweep (global override) on the ResNet-50 bench
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05z; mkdir -p $O
python -c "import sys; sys.path.insert(0, '.'); import hyperion._C as m; assert hasattr(m, 'conv_set_group')" || exit 1
for g in 0 -1 -2 4 8 16 1 0; do
  HYPERION_CONV_GROUP=$g timeout -k 10 150 python bench.py --steps 50 --warmup 10 > $O/b.json 2>>$O/err || exit 1
  python -c "import json; print('group $g', json.load(open('$O/b.json'))['ms_per_step'])"
done
