#!/bin/bash
# round 5: compile-time 3x3/s2 max pool (all taps' loads in flight) — tests, bench A/B, per-kernel times
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05mp; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pool.py tests/test_gpu_round4.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench$i.log 2>&1 || { tail -5 $O/bench$i.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/bench$i.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof" -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); grep -i "maxpool" "$f" | cut -c1-200
