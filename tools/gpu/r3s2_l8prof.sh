# steady-state kernel stats of the Llama-3-8B bench on the final kernels
set -o pipefail
mkdir -p gpurun_out/l8p
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
AKAP_GEMM_TUNE_CACHE=/tmp/tl.json timeout -k 10 500 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/l8p/warm.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tl.json timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/l8p/prof -o run -- python3 bench.py --model llama-3-8b --steps 1 --warmup 1 > gpurun_out/l8p/prof.log 2>&1
