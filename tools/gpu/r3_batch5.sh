# round 3, batch 5: the engine's two-micro-batch decode (AKAP_UBATCH=1: the real fused chain per
# half, free-running on two streams in one hipGraph) with the grid-capped persistent attention
set -o pipefail
mkdir -p gpurun_out/ov
AKAP_UBATCH=1 AKAP_ATTN_FLAGS=73 timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ov/ub_f73.log 2>&1 && \
AKAP_UBATCH=1 AKAP_ATTN_FLAGS=81 timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ov/ub_f81.log 2>&1 && \
AKAP_UBATCH=1 AKAP_ATTN_FLAGS=65 timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ov/ub_f65.log 2>&1
