# 256-row decode GEMM with the half-step pipelined K loop (AKAP_GDGEMM_PIPE=1): numerics, M=256
# sweep A/B (Llama-3-8B + 70B shard shapes), Llama-3-8B bench A/B
set -o pipefail
mkdir -p gpurun_out/gp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
AKAP_GDGEMM_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "lds_dma_decode_gemm and rows256" > gpurun_out/gp/tests.log 2>&1 && \
AKAP_GDGEMM_PIPE=1 timeout -k 10 300 python -u tools/gemm_m256.py --only llama8b > gpurun_out/gp/sweep_pipe.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_m256.py --only llama8b > gpurun_out/gp/sweep_base.log 2>&1 && \
AKAP_GDGEMM_PIPE=1 timeout -k 10 300 python -u tools/gemm_m256.py --only llama70b_tp8 > gpurun_out/gp/sweep70_pipe.log 2>&1 && \
AKAP_GDGEMM_PIPE=1 timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/gp/llama8b_pipe.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/gp/llama8b_base.log 2>&1
