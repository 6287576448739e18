# round 3, batch 12: prefill attention tile size for the headline's 512-token prompts
set -o pipefail
mkdir -p gpurun_out/tr
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/tr/t128.log 2>&1 && \
AKAP_PREFILL_TILE_ROWS=256 AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/tr/t256.log 2>&1 && \
AKAP_PREFILL_TILE_ROWS=64 AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/tr/t64.log 2>&1
