# prologue operand loads with shared addresses for lanes that do not need them: numerics + bench
set -o pipefail
mkdir -p gpurun_out/ln
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "decode or v_tail" > gpurun_out/ln/tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ln/engine.log 2>&1 && \
timeout -k 10 200 python -u bench/attn_fused_ab.py > gpurun_out/ln/fused_ab.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ln/bench_a.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ln/bench_b.log 2>&1
