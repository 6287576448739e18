# round 3, batch 13: Llama-3-8B steady-state kernel stats (P/D headline model, decode anatomy)
set -o pipefail
mkdir -p gpurun_out/l8
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
AKAP_GEMM_TUNE_CACHE=/tmp/tune8.json timeout -k 10 500 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/l8/warm.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune8.json timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/l8/prof -o run -- python3 bench.py --model llama-3-8b --steps 1 --warmup 1 > gpurun_out/l8/prof.log 2>&1
