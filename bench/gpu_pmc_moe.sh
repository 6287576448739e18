# PMC passes of the Mixtral MoE block (bench/pmc_targets.py --mode moe); see gpu_pmc_passes.sh
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
P1="FETCH_SIZE SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
set -e
timeout -s KILL 150 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc_moe_1 -o run -- python3 bench/pmc_targets.py --mode moe --iters 5 > gpurun_out/pmc_moe_1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmc_moe_2 -o run -- python3 bench/pmc_targets.py --mode moe --iters 5 > gpurun_out/pmc_moe_2.log 2>&1
echo moe ok
