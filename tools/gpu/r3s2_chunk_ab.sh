# prefill chunk size (max_num_batched_tokens) A/B on the headline workload, Qwen3-0.6B and Llama-3-8B
set -o pipefail
mkdir -p gpurun_out/ck
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
AKAP_GEMM_TUNE_CACHE=/tmp/tq.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ck/q_16k.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tq.json timeout -k 10 300 python -u bench.py --steps 2 --max-num-batched-tokens 32768 > gpurun_out/ck/q_32k.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tq.json timeout -k 10 300 python -u bench.py --steps 2 --max-num-batched-tokens 65536 > gpurun_out/ck/q_64k.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tl.json timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/ck/l_16k.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tl.json timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 1 --max-num-batched-tokens 32768 > gpurun_out/ck/l_32k.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tl.json timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 1 --max-num-batched-tokens 8192 > gpurun_out/ck/l_8k.log 2>&1
