#!/bin/bash
# Full GPU check: smoke, every GPU test, ResNet-50 bench, model suite (LM / ViT / Llama / fusion).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "[$n] $(date +%T) start"; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "[$n] rc=$rc"; grep -E "passed|failed|^\{" gpurun_out/$n.log | cut -c1-300 | tail -4; if [ $rc -ne 0 ]; then tail -40 gpurun_out/$n.log; exit $rc; fi; }
run smoke 300 python3 __graft_entry__.py smoke
run pytest_gpu 600 python3 -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread
run bench_graph 300 python3 bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench_graph.json
run models 900 python3 -m hyperion.cli.bench_models --out gpurun_out/models --only ${MODELS:-lm,vit,llama,fusion}
echo done
