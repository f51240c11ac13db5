#!/bin/bash
# round 5, call T: PMC passes on the native GEMM (gpt2 out_proj 2032x768x768, 64x128 tile) and the
# vendor GEMM of the same shape — where the k-loop waits
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$PWD/gpurun_out/r05t; mkdir -p $O
P="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
for v in "2032 768 768 6 1 native" "2032 768 768 2 1 native" "2032 768 768 2 1 vendor" "2032 3072 768 6 1 native" "2032 3072 768 6 1 vendor"; do
  set -- $v
  tag=$1x$2x$3_t$4_$6
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$tag -o run -- python3 $PWD/scripts/micro/gemm_one.py $v > $O/pmc_$tag.log 2>&1 || { tail -5 $O/pmc_$tag.log; exit 1; }
  echo "$tag done"
done
python3 - <<PY
import csv, glob, collections
for d in sorted(glob.glob('$O/pmc_*')):
    fs = glob.glob(d + '/**/*counter_collection.csv', recursive=True)
    if not fs: continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(fs[0])):
        k = r['Kernel_Name'][:60]
        if 'gemm' not in k and 'Cijk' not in k: continue
        agg[k][r['Counter_Name']] += float(r['Counter_Value']); n[(k, r['Counter_Name'])] += 1
    for k, c in agg.items():
        calls = max(n[(k, 'SQ_WAVES')], 1)
        wc = c['SQ_WAVE_CYCLES'] or 1
        print(d.split('/')[-1], k[:50], 'calls', calls, {kk: round(v / calls) for kk, v in c.items()},
              'wait_any %.2f wait_inst %.2f active %.2f' % (c['SQ_WAIT_ANY'] / wc, c['SQ_WAIT_INST_ANY'] / wc, c['SQ_ACTIVE_INST_ANY'] / wc))
PY
