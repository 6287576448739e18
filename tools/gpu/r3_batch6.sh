# round 3, batch 6: V tail (decode writes whole 8-token V groups) -- kernel numerics, engine
# end-to-end tests, headline bench with and without it
set -o pipefail
mkdir -p gpurun_out/vt
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "v_tail or decode or qk_norm_rope_cache" > gpurun_out/vt/kern.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/vt/engine.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/vt/bench_tail.log 2>&1 && \
AKAP_V_TAIL=0 timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/vt/bench_notail.log 2>&1
