set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_decode.py tests/test_kernels_gpu.py -k "fused or tuner or lds_dma" > gpurun_out/dgemm_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 2 > gpurun_out/bench_llama8b.log 2>&1
