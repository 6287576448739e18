# round 3, batch 15: 32-bit index math in the reduce / combine / embedding kernels -- numerics,
# then the Llama-3-8B and Qwen3 benches with kernel stats for Llama
set -o pipefail
mkdir -p gpurun_out/l8c
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/l8c/tests.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune8.json timeout -k 10 500 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/l8c/warm.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune8.json timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/l8c/prof -o run -- python3 bench.py --model llama-3-8b --steps 1 --warmup 1 > gpurun_out/l8c/prof.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/l8c/qwen3.log 2>&1
