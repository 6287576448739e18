# round 3, batch 7: P/D hand-off with the V tail on the GPU; steady-state kernel stats of the
# headline bench (tuning cache written by a first, unprofiled run); Llama-3-8B bench
set -o pipefail
mkdir -p gpurun_out/b7
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -k "pd_handoff" > gpurun_out/b7/pd_tail.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 1 > gpurun_out/b7/bench_warm.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b7/prof -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/b7/bench_prof.log 2>&1 && \
timeout -k 10 500 python -u bench.py --model llama-3-8b --steps 1 > gpurun_out/b7/llama8b.log 2>&1
