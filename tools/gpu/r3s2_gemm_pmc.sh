# PMC passes on the 256-row decode GEMM (Llama-3-8B gate_up, M = 256), one counter group per run
set -o pipefail
mkdir -p gpurun_out/gpmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python -u tools/gemm_pmc_probe.py > gpurun_out/gpmc/plain.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/gpmc/p1 -o run -- python3 tools/gemm_pmc_probe.py > gpurun_out/gpmc/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM_RD GRBM_COUNT --output-format csv -d gpurun_out/gpmc/p2 -o run -- python3 tools/gemm_pmc_probe.py > gpurun_out/gpmc/p2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TA_BUSY_avr TD_BUSY_avr --output-format csv -d gpurun_out/gpmc/p3 -o run -- python3 tools/gemm_pmc_probe.py > gpurun_out/gpmc/p3.log 2>&1
