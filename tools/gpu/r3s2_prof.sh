# steady-state kernel stats of the headline bench (tuning cache written by a first, unprofiled run)
set -o pipefail
mkdir -p gpurun_out/p1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 1 > gpurun_out/p1/bench_warm.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p1/prof -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/p1/bench_prof.log 2>&1
