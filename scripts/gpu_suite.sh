#!/bin/bash
# One-GPU measurement suite (run through gpurun or on any MI355X box); every step has its own time
# limit and a failing step ends the run.  Output under gpurun_out/suite/<stage>/.
#
#   bash scripts/gpu_suite.sh tests [pytest files ...]   GPU tests (default: every tests/test_gpu_*.py)
#   bash scripts/gpu_suite.sh bench                      ResNet-50 bench.py, 50 timed steps
#   bash scripts/gpu_suite.sh trace                      rocprofv3 kernel trace of the bench step (+ step table)
#   bash scripts/gpu_suite.sh tune                       conv launch-plan tuning (HBM-cold) + A/B bench kept vs new
#   bash scripts/gpu_suite.sh timeline                   per-workgroup conv timelines (diagnostic stamps)
#   bash scripts/gpu_suite.sh models                     LM-256 / GPT-2 / ViT graphed steps (+ DDP at world 1)
#   bash scripts/gpu_suite.sh fsdp                       FSDP steps: LM-256 / GPT-2 graphed, GPT-2 reshard, Llama-7B full
#   bash scripts/gpu_suite.sh lmhead                     LM-head + CE schedules, GEMM epilogue probe
#   bash scripts/gpu_suite.sh baseline                   reference-methodology model benchmarks + fused-vs-eager
#   bash scripts/gpu_suite.sh pmc                        PMC counter passes over ResNet-50 steps -> per-kernel table
#   bash scripts/gpu_suite.sh rccl                       RCCL reduce-scatter / all-reduce tail check
#   bash scripts/gpu_suite.sh gemm                       native GEMM tiles (classic + ping-pong) vs vendor sweep
#   bash scripts/gpu_suite.sh gemm_pmc                   PMC passes over single GEMM shapes (native vs vendor)
#   bash scripts/gpu_suite.sh llama_pmc                  PMC passes over the Llama-2-7B LoRA step (weight streaming)
#   bash scripts/gpu_suite.sh steps                      graphed model steps (WL="vitgraph vitselgraph ..."), one JSON each
#   bash scripts/gpu_suite.sh final                      bench x2 + every README step row (one box, one call)
#   bash scripts/gpu_suite.sh refresh                    README micro rows: matmul / STREAM, attention, LM head, fused-vs-eager
#   bash scripts/gpu_suite.sh fp32                       fp32 path: three-loop rows native vs vendor, fp32 GEMM vs hipBLASLt, routes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
stage=${1:-bench}
shift || true
out=gpurun_out/suite/$stage
mkdir -p "$out"

json_ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1; }

case $stage in
tests)
  files=${*:-tests/test_gpu_*.py}
  timeout -k 10 1500 python -u -m pytest -x -q --timeout 300 --timeout-method thread $files > "$out/pytest.log" 2>&1
  rc=$?; tail -3 "$out/pytest.log"; exit $rc
  ;;
bench)
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > "$out/bench.json" 2> "$out/bench.err" || exit 1
  json_ms "$out/bench.json"
  ;;
trace)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$out/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" || exit 1
  f=$(ls "$out"/prof/*/run_kernel_trace.csv 2>/dev/null || ls "$out"/prof/run_kernel_trace.csv) || exit 1
  python3 scripts/step_trace.py "$f" --step -2 --out "$out/step.txt" > /dev/null && \
  python3 scripts/kstats.py "$f" > "$out/kstats.txt" 2>&1 || exit 1
  grep -E "step -2" "$out/step.txt"; head -20 "$out/kstats.txt" | cut -c1-160
  ;;
tune)
  timeout -k 10 1000 python -u scripts/conv_tune.py --out "$out/conv_plans.json" --raw "$out/conv_tune_raw.json" \
    > "$out/conv_tune.log" 2>&1 || exit 1
  tail -5 "$out/conv_tune.log"
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > "$out/bench_kept.json" 2>/dev/null && \
  HYPERION_CONV_PLANS=$PWD/$out/conv_plans.json timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 \
    > "$out/bench_new.json" 2>/dev/null || exit 1
  echo kept $(json_ms "$out/bench_kept.json"); echo new $(json_ms "$out/bench_new.json")
  ;;
timeline)
  timeout -k 10 200 python -u scripts/conv_timeline.py --out "$out/timeline.json" > "$out/timeline.log" 2>&1 || exit 1
  tail -12 "$out/timeline.log" | cut -c1-200
  ;;
models)
  for w in ${WL:-lmgraph gpt2 vitgraph lmddp1g vitddp1g}; do
    timeout -k 10 300 python -u scripts/run_model_step.py $w > "$out/$w.json" 2> "$out/$w.err" || { tail -5 "$out/$w.err"; exit 1; }
    echo $w $(json_ms "$out/$w.json")
  done
  ;;
fsdp)
  for cfg in "lm256 graph" "gpt2_small graph" "gpt2_small reshard" "gpt2_small graph coll" "llama7b_full curve"; do
    timeout -k 10 400 python -u scripts/run_model_step.py fsdp $cfg >> "$out/fsdp_steps.jsonl" 2>> "$out/fsdp_steps.err" || exit 1
  done
  grep "^{" "$out/fsdp_steps.jsonl" | cut -c1-260
  ;;
lmhead)
  timeout -k 10 300 python -u scripts/ce_bench.py --out "$out/ce_bench.json" > "$out/ce_bench.log" 2>&1 && \
  timeout -k 10 300 python -u scripts/gemm_probe.py --out "$out/gemm_probe.json" > "$out/gemm_probe.log" 2>&1 || exit 1
  grep -v amdgpu.ids "$out/ce_bench.log" | cut -c1-300
  ;;
baseline)
  # the reference-methodology ResNet / CNN benchmark (fp32, torch and Hyperion kernels; bf16) and the
  # fused-vs-eager inference study
  PYTHONPATH=$PWD timeout -k 10 900 python -u -m hyperion.cli.bench_models --out "$out" --only baseline,fusion \
    > "$out/bench_models.log" 2>&1 || { tail -20 "$out/bench_models.log"; exit 1; }
  ls "$out"; tail -5 "$out/bench_models.log"
  ;;
pmc)
  # counter passes (one run each, no tracing) over eager ResNet-50 bench steps -> per-kernel table
  P1="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_LDS_BANK_CONFLICT,GRBM_GUI_ACTIVE"
  P2="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_MFMA,SQ_WAVES,SQ_INST_LEVEL_VMEM,SQ_WAIT_INST_LDS,GRBM_GUI_ACTIVE"
  P3="TCC_HIT_sum,TCC_MISS_sum,GRBM_GUI_ACTIVE"
  P4="FETCH_SIZE,GRBM_GUI_ACTIVE"
  P5="WRITE_SIZE,GRBM_GUI_ACTIVE"
  i=0
  for pass in "$P1" "$P2" "$P3" "$P4" "$P5"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d "$PWD/$out/resnet50_P$i" -o run -- \
      python3 bench.py --graph 0 --steps 3 --warmup 2 > "$out/pass_$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$out/pass_$i.log"; exit 1; }
    f=$(ls "$out"/resnet50_P$i/*/run_counter_collection.csv 2>/dev/null | head -1)
    [ -n "$f" ] && cp "$f" "$out/resnet50_P$i/run_counter_collection.csv"
  done
  python3 scripts/pmc_summary.py "$out" --out "$out/pmc_table.md" > /dev/null || exit 1
  head -30 "$out/pmc_table.md" | cut -c1-260
  ;;
rccl)
  timeout -k 10 200 python -u scripts/rccl_avg_check.py > "$out/rccl.log" 2>&1 || exit 1
  grep -E "^bad|^rs" "$out/rccl.log"
  ;;
gemm)
  timeout -k 10 600 python -u scripts/gemm_pp_sweep.py --big > "$out/sweep.jsonl" 2> "$out/sweep.err" || { tail -5 "$out/sweep.err"; exit 1; }
  python3 scripts/gemm_sweep_summary.py "$out/sweep.jsonl"
  ;;
gemm_pmc)
  bash scripts/gemm_pmc.sh "$out"
  ;;
llama_pmc)
  bash scripts/llama_pmc.sh "$out"
  ;;
steps)
  for w in ${WL:-vitgraph vitselgraph vitckptgraph gpt2 lmgraph llamagraph}; do
    timeout -k 10 400 python -u scripts/run_model_step.py $w > "$out/$w.json" 2> "$out/$w.err" || { echo "[$w] FAILED"; tail -5 "$out/$w.err"; exit 1; }
    python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(r['ms_per_step'],3), 'ms, peak', round(r.get('peak_mem_mb',0)), 'MB')" "$out/$w.json" $w
  done
  ;;
steptrace)
  # kernel trace of one graphed model step per workload (WL): per-step kernel table + vendor-GEMM count
  export HSA_ENABLE_IPC_MODE_LEGACY=0
  for w in ${WL:-vitgraph gpt2}; do
    rm -rf "$out/raw_$w"
    timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$out/raw_$w" -o run -- \
      python3 scripts/run_model_step.py $w > "$out/$w.json" 2> "$out/$w.err" || { echo "[$w] trace failed"; tail -5 "$out/$w.err"; exit 1; }
    f=$(find "$out/raw_$w" -name "*kernel_trace.csv" | head -1)
    python3 scripts/step_trace.py "$f" --step -2 --out "$out/step_$w.txt" > /dev/null || exit 1
    rm -rf "$out/raw_$w"
    echo "$w: $(grep -E '^step' "$out/step_$w.txt") vendor GEMM kernels: $(grep -c 'Cijk' "$out/step_$w.txt")"
  done
  ;;
final)
  # the README's measured rows from ONE box: bench.py x2 (driver contract), DDP at world 1, graphed
  # model steps, FSDP steps (ring / persistent, with the native collectives at world 1)
  export HSA_ENABLE_IPC_MODE_LEGACY=0
  for i in 1 2; do
    timeout -k 10 300 python -u bench.py > "$out/bench$i.json" 2> "$out/bench$i.err" || { tail -5 "$out/bench$i.err"; exit 1; }
    echo "bench$i $(json_ms "$out/bench$i.json")"
  done
  timeout -k 10 300 python -u bench.py --ddp-world1 1 > "$out/bench_ddp1.json" 2> "$out/bench_ddp1.err" || { tail -5 "$out/bench_ddp1.err"; exit 1; }
  echo "bench_ddp1 $(json_ms "$out/bench_ddp1.json")"
  for w in ${WL:-vitgraph vitselgraph vitckptgraph gpt2 lmgraph llamagraph20}; do
    timeout -k 10 400 python -u scripts/run_model_step.py $w > "$out/$w.json" 2> "$out/$w.err" || { echo "[$w] FAILED"; tail -5 "$out/$w.err"; exit 1; }
    echo "$w $(json_ms "$out/$w.json")"
  done
  for cfg in "gpt2_small graph ring3 coll" "gpt2_small graph coll" "gpt2_small graph ring3" "lm256 graph coll"; do
    timeout -k 10 400 python -u scripts/run_model_step.py fsdp $cfg >> "$out/fsdp_steps.jsonl" 2>> "$out/fsdp_steps.err" || { tail -5 "$out/fsdp_steps.err"; exit 1; }
    echo "fsdp $cfg $(tail -1 "$out/fsdp_steps.jsonl" | grep -o '"ms_per_step": [0-9.]*')"
  done
  ;;
refresh)
  PYTHONPATH=$PWD timeout -k 10 500 python -u -m hyperion.cli.hardware_bench --out "$out/hardware" > "$out/hardware.log" 2>&1 || { tail -5 "$out/hardware.log"; exit 1; }
  echo hardware ok
  timeout -k 10 300 python -u scripts/attn_bench.py > "$out/attn_bench.jsonl" 2> "$out/attn_bench.err" || { tail -5 "$out/attn_bench.err"; exit 1; }
  echo attn ok
  timeout -k 10 300 python -u scripts/ce_bench.py --out "$out/ce_bench.json" > "$out/ce_bench.log" 2>&1 || { tail -5 "$out/ce_bench.log"; exit 1; }
  echo ce ok
  PYTHONPATH=$PWD timeout -k 10 400 python -u -m hyperion.cli.bench_models --out "$out/fusion/x" --only fusion > "$out/fusion.log" 2>&1 || { tail -5 "$out/fusion.log"; exit 1; }
  ls "$out" "$out/hardware" "$out/fusion"
  ;;
fp32)
  timeout -k 10 300 python -u scripts/fp32_step.py create_resnet50 1 10 > "$out/routes.txt" 2>&1 || { tail -5 "$out/routes.txt"; exit 1; }
  timeout -k 10 600 python -u scripts/fp32_ab.py > "$out/three_loop_ab.jsonl" 2> "$out/three_loop_ab.err" || { tail -5 "$out/three_loop_ab.err"; exit 1; }
  timeout -k 10 300 python -u scripts/f32_gemm_probe.py --short > "$out/gemm_probe.jsonl" 2> "$out/gemm_probe.err" || exit 1
  head -3 "$out/routes.txt"; cut -c1-160 "$out/three_loop_ab.jsonl"
  ;;
*)
  echo "unknown stage $stage"; exit 2
  ;;
esac
