# fused decode attention: new token's K/V patched from LDS images (no cache store drain):
# numerics, fused-variant breakdown micro, headline bench, engine tests
set -o pipefail
mkdir -p gpurun_out/ki
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "decode or v_tail" > gpurun_out/ki/tests.log 2>&1 && \
timeout -k 10 200 python -u bench/attn_fused_ab.py > gpurun_out/ki/fused_ab.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ki/engine.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ki/bench_a.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ki/bench_b.log 2>&1
