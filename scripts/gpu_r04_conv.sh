set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/conv_roofline.py --out gpurun_out/r04/conv_roofline.json > gpurun_out/r04/conv_roofline.log 2>&1 && \
P1="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_LDS_BANK_CONFLICT,GRBM_GUI_ACTIVE" && \
P2="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_MFMA,SQ_WAVES,SQ_INST_LEVEL_VMEM,SQ_WAIT_INST_LDS,GRBM_GUI_ACTIVE" && \
i=0 && for shape in "32 256 14 256 3 1 1" "32 64 56 64 3 1 1"; do
  for pass in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$PWD/gpurun_out/r04/pmc/p$i" -o run -- python3 "$PWD/scripts/conv_one.py" $shape > gpurun_out/r04/pmc_$i.log 2>&1 || exit 1
  done
done
echo done
