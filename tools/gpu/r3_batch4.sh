# round 3, batch 4: two-micro-batch decode overlap with a grid-capped (persistent) fused decode
# attention, so the other half's GEMMs find free CU slots; MoE grouped-path GPU test
set -o pipefail
mkdir -p gpurun_out/ov
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "moe" > gpurun_out/ov/moe_tests.log 2>&1 && \
AKAP_ATTN_FLAGS=65 OVERLAP_SYNC=none timeout -k 10 240 python -u bench/overlap_micro.py > gpurun_out/ov/f65.log 2>&1 && \
AKAP_ATTN_FLAGS=73 OVERLAP_SYNC=none timeout -k 10 240 python -u bench/overlap_micro.py > gpurun_out/ov/f73.log 2>&1 && \
AKAP_ATTN_FLAGS=81 OVERLAP_SYNC=none timeout -k 10 240 python -u bench/overlap_micro.py > gpurun_out/ov/f81.log 2>&1 && \
AKAP_ATTN_FLAGS=89 OVERLAP_SYNC=none timeout -k 10 240 python -u bench/overlap_micro.py > gpurun_out/ov/f89.log 2>&1
