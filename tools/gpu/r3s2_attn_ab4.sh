# decode attention: barrier-free fused prologue (default) vs the workgroup prologue (bit 9):
# numerics, fused-vs-plain micro, headline bench A/B, kernel stats
set -o pipefail
mkdir -p gpurun_out/ab4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "decode or v_tail" > gpurun_out/ab4/tests.log 2>&1 && \
timeout -k 10 120 python -u bench/attn_fused_ab.py > gpurun_out/ab4/fused_ab.log 2>&1 && \
AKAP_ATTN_FLAGS=577 timeout -k 10 120 python -u bench/attn_fused_ab.py > gpurun_out/ab4/fused_ab_577.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab4/bench_65.log 2>&1 && \
AKAP_ATTN_FLAGS=577 AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab4/bench_577.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab4/bench_65b.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab4/engine_tests.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab4/prof -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/ab4/bench_prof.log 2>&1
