#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-p16}
mkdir -p gpurun_out/r04/$tag
for w in ${WL:-lmgraph lmddp1 vitgraph vitddp1}; do
  timeout -k 10 300 python -u scripts/run_model_step.py $w > gpurun_out/r04/$tag/$w.json 2> gpurun_out/r04/$tag/$w.err || { echo "$w failed"; tail -5 gpurun_out/r04/$tag/$w.err; exit 1; }
  echo $w $(grep -o '"ms_per_step": [0-9.]*\|"buckets": [0-9]*\|"comm": "[A-Za-z]*"' gpurun_out/r04/$tag/$w.json | tr '\n' ' ')
done
[ -n "$NOTRACE" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/r04/$tag/prof" -o run -- python3 scripts/run_model_step.py gpt2 > gpurun_out/r04/$tag/gpt2.json 2>/dev/null && \
python3 scripts/kstats.py $(ls gpurun_out/r04/$tag/prof/run_kernel_trace.csv gpurun_out/r04/$tag/prof/*/run_kernel_trace.csv 2>/dev/null | head -1) 60 0.5 > gpurun_out/r04/$tag/gpt2_kstats.txt
echo trace rc=$?; grep -c "dropout_k\|GeluCUDA" gpurun_out/r04/$tag/gpt2_kstats.txt || true; head -3 gpurun_out/r04/$tag/gpt2_kstats.txt | cut -c1-150
