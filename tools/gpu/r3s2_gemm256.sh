# 256-row decode GEMM: 6-slot ring of 32-deep k-steps vs the 3-slot 64-deep ring: numerics,
# M=256 sweep (8B / 70B-shard / Qwen3 shapes, cold weights), Llama-3-8B bench
set -o pipefail
mkdir -p gpurun_out/g256
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "lds_dma_decode_gemm" > gpurun_out/g256/tests.log 2>&1 && \
timeout -k 10 400 python -u tools/gemm_m256.py > gpurun_out/g256/sweep.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/g256/llama8b.log 2>&1
