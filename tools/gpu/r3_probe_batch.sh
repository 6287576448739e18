set -o pipefail
mkdir -p gpurun_out/obs gpurun_out/pmc_cal
AKAP_UBATCH=0 timeout -k 10 240 python -u bench.py --steps 2 > gpurun_out/ubatch0.log 2>&1 && \
AKAP_UBATCH=1 timeout -k 10 240 python -u bench.py --steps 2 > gpurun_out/ubatch1.log 2>&1 && \
export AKAP_GEMM_TUNE_CACHE=/tmp/akap_tune_cal.json && \
timeout -k 10 240 python -u tools/pmc_calibrate.py > gpurun_out/pmc_cal/workload_plain.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_cal -o run -- python3 tools/pmc_calibrate.py > gpurun_out/pmc_cal/workload_pmc.log 2>&1 && \
unset AKAP_GEMM_TUNE_CACHE && \
timeout -k 10 400 python -u tools/observability_probe.py > gpurun_out/obs/probe.log 2>&1
