# non-temporal weight DMA (AKAP_WEIGHT_NT=1) A/B on the decode GEMMs: numerics, Qwen3 + Llama-3-8B
# benches (same GEMM plan: the tuning cache written by the first, default-policy run)
set -o pipefail
mkdir -p gpurun_out/nt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
AKAP_WEIGHT_NT=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "lds_dma_decode_gemm or kgemm" > gpurun_out/nt/tests.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tq.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/nt/q_base.log 2>&1 && \
AKAP_WEIGHT_NT=1 AKAP_GEMM_TUNE_CACHE=/tmp/tq.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/nt/q_nt.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tl.json timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/nt/l_base.log 2>&1 && \
AKAP_WEIGHT_NT=1 AKAP_GEMM_TUNE_CACHE=/tmp/tl.json timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/nt/l_nt.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tl.json timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/nt/l_base2.log 2>&1 && \
AKAP_WEIGHT_NT=1 AKAP_GEMM_TUNE_CACHE=/tmp/tl.json timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/nt/l_nt2.log 2>&1
