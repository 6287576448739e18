# round 3, batch 2: observability probe, MoE prefill paths, Llama-3-70B TP=8 rank rehearsal and
# Llama-3-8B 1-GPU bench with the 256-row GEMM tiles in the tuner
set -o pipefail
mkdir -p gpurun_out/obs
timeout -k 10 400 python -u tools/observability_probe.py > gpurun_out/obs/probe.log 2>&1 && \
timeout -k 10 300 python -u tools/moe_prefill.py > gpurun_out/moe_prefill.log 2>&1 && \
timeout -k 10 400 python -u bench/tp_shard_rehearsal.py > gpurun_out/tp8_rehearsal.log 2>&1 && \
timeout -k 10 500 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/llama8b_bench.log 2>&1
