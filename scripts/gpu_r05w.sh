#!/bin/bash
# round 5, call W: BN apply / dx pass grid sweep (row-block cap, min row iterations) on the bench
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bn_adam.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
python -c "import sys; sys.path.insert(0, '.'); import hyperion._C as m; assert hasattr(m, 'bn_set_geom')" || exit 1
for g in default 1024,4 2048,2 4096,2 4096,4 8192,1 8192,2 2048,8 default; do
  if [ $g = default ]; then
    timeout -k 10 150 python bench.py --steps 50 --warmup 10 > $O/b.json 2>>$O/err || exit 1
  else
    HYPERION_BN_GEOM=$g timeout -k 10 150 python bench.py --steps 50 --warmup 10 > $O/b.json 2>>$O/err || exit 1
  fi
  python -c "import json; print('$g', json.load(open('$O/b.json'))['ms_per_step'])"
done
