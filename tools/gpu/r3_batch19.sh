# round 3, batch 19: in-process kernel-stats windows on hardware -- the engine GPU test and the
# real server under HTTP load serving akap_kernel_* on its own /metrics
set -o pipefail
mkdir -p gpurun_out/obs2
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "inprocess" > gpurun_out/obs2/test.log 2>&1 && \
timeout -k 10 400 python -u tools/observability_probe.py --out gpurun_out/obs2 --inprocess > gpurun_out/obs2/probe.log 2>&1
