# round-3 session-2: GPU suite + smoke + decode-attention micro + 1-GPU benches (each step
# time-limited; stop at the first failure)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 120 python -u bench/attn_micro.py --B 256 --ctx 640 --spread 0 --parts 1 > gpurun_out/attn_micro.log 2>&1 && \
timeout -k 10 120 python -u bench/attn_micro.py --B 32 --ctx 2048 --spread 0 --parts 1 >> gpurun_out/attn_micro.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 2 > gpurun_out/bench_llama8b.log 2>&1
