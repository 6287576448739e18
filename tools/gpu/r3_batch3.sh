# round 3, batch 3: 256-row gdgemm tiles vs fp32 references, MoE prefill paths (incl.
# torch._grouped_mm), Llama-3-70B TP=8 rank rehearsal with the real all-reduce kernels, the
# Qwen3 headline bench with the LM head candidates, amd-smi list schema
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "lds_dma_decode_gemm" > gpurun_out/gdgemm256_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/moe_prefill.py > gpurun_out/moe_prefill.log 2>&1 && \
timeout -k 10 400 python -u bench/tp_shard_rehearsal.py > gpurun_out/tp8_rehearsal.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/qwen3_bench_r3d.log 2>&1 && \
timeout -k 10 60 /opt/rocm/bin/amd-smi list --json > gpurun_out/amdsmi_list.json 2>&1
