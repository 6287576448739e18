# round 3, batch 14: row-parallel rmsnorm + 32-bit silu_and_mul indexing -- numerics, then the
# Llama-3-8B bench and its kernel stats
set -o pipefail
mkdir -p gpurun_out/l8b
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "rmsnorm or silu" > gpurun_out/l8b/kern.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune8.json timeout -k 10 500 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/l8b/warm.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune8.json timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/l8b/prof -o run -- python3 bench.py --model llama-3-8b --steps 1 --warmup 1 > gpurun_out/l8b/prof.log 2>&1
