set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "moe or mixtral" > gpurun_out/moe_tests.log 2>&1 && \
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --num-requests 128 --steps 1 > gpurun_out/bench_mixtral.log 2>&1
