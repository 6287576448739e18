set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_decode.py tests/test_kernels_gpu.py -k "fused or tuner" > gpurun_out/dgemm_tests.log 2>&1 && \
timeout -k 10 300 python -u bench/fused_chain_micro.py > gpurun_out/fused_chain_micro.log 2>&1 && \
timeout -k 10 300 python -u bench/dgemm_micro.py --m 256 --pfs 4,8 --splits 1,2,4 > gpurun_out/dgemm_micro_qwen.log 2>&1
