# round 3, batch 16: row-parallel RESNORM split-K reduce -- numerics (gdgemm epilogue tests +
# fused decode tests + engine), then Llama-3-8B bench + kernel stats
set -o pipefail
mkdir -p gpurun_out/l8d
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/l8d/tests.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune8.json timeout -k 10 500 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/l8d/warm.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune8.json timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/l8d/prof -o run -- python3 bench.py --model llama-3-8b --steps 1 --warmup 1 > gpurun_out/l8d/prof.log 2>&1
