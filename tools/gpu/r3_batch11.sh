# round 3, batch 11: side-stream MALL prefetch of the decode GEMM weights (AKAP_SIDE_PREFETCH=1):
# captures? numerics (engine GPU tests)? bench + kernel stats vs off
set -o pipefail
mkdir -p gpurun_out/sp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
AKAP_SIDE_PREFETCH=1 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sp/engine.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/sp/off.log 2>&1 && \
AKAP_SIDE_PREFETCH=1 AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/sp/on.log 2>&1 && \
AKAP_SIDE_PREFETCH=1 AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp/prof -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/sp/prof.log 2>&1
