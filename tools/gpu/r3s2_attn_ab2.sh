# decode attention: 3-workgroups-per-CU single-buffered variant vs the default, numerics + bench
set -o pipefail
mkdir -p gpurun_out/ab2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "persistent_variants" > gpurun_out/ab2/tests.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab2/bench_65.log 2>&1 && \
AKAP_ATTN_FLAGS=321 AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab2/bench_321.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab2/bench_65b.log 2>&1 && \
AKAP_ATTN_FLAGS=321 AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab2/bench_321b.log 2>&1 && \
timeout -k 10 120 python -u bench/attn_fused_ab.py > gpurun_out/ab2/fused_ab.log 2>&1
