# decode-attention variants: numerics (persistent / pipelined), then the headline bench per
# variant (same box, back to back, shared GEMM tuning cache), then steady-state kernel stats
set -o pipefail
mkdir -p gpurun_out/ab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "decode" > gpurun_out/ab/tests.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab/bench_65.log 2>&1 && \
AKAP_ATTN_FLAGS=209 AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab/bench_209.log 2>&1 && \
AKAP_ATTN_FLAGS=81 AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab/bench_81.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab/bench_65b.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/prof -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/ab/bench_prof.log 2>&1 && \
AKAP_ATTN_FLAGS=209 AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/prof209 -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/ab/bench_prof209.log 2>&1
