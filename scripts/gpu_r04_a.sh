#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
tag=${1:-a}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_round4.py tests/test_gpu_conv.py tests/test_gpu_llm_ops.py > gpurun_out/r04/pytest_$tag.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/r04/bench_$tag.json 2> gpurun_out/r04/bench_$tag.err && \
timeout -k 10 200 python -u scripts/conv_timeline.py --out gpurun_out/r04/timeline_$tag.json > gpurun_out/r04/timeline_$tag.log 2>&1 && \
bash scripts/gpu_r04_trace.sh trace_$tag > /dev/null 2>&1
echo rc=$?
tail -3 gpurun_out/r04/pytest_$tag.log; cut -c1-150 gpurun_out/r04/bench_$tag.json; grep -E "step -2" gpurun_out/r04/trace_$tag/step.txt
python3 - <<'PY' "$tag"
import json,sys
for r in json.load(open(f"gpurun_out/r04/timeline_{sys.argv[1]}.json")):
    print(r["op"], r["C"], r["H"], r["K"], r["R"], "span", r["span_us"], "pro", r["prologue_us_med"], "loop", r["loop_us_med"], "epi", r["epilogue_us_med"], "conc", r["max_concurrent_per_cu"])
PY
if [ "${TUNE:-0}" = "1" ]; then
  timeout -k 10 1000 python -u scripts/conv_tune.py --out gpurun_out/r04/conv_plans_$tag.json --raw gpurun_out/r04/conv_tune_raw_$tag.json > gpurun_out/r04/conv_tune_$tag.log 2>&1
  echo tune rc=$?; tail -1 gpurun_out/r04/conv_tune_$tag.log
fi
