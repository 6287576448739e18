# PMC passes (2 counter groups each) over the decode and prefill targets, one run per pass.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
P1="FETCH_SIZE SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
set -e
for mode in decode prefill; do
  for pass in 1 2; do
    if [ $pass = 1 ]; then C="$P1"; else C="$P2"; fi
    timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcb_${mode}_${pass} -o run -- python3 bench/pmc_targets.py --mode $mode --iters 5 > gpurun_out/pmcb_${mode}_${pass}.log 2>&1
    echo "pass $mode $pass ok"
  done
done
