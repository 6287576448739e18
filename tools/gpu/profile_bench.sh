# rocprofv3 kernel-trace + stats of the headline bench (1 timed wave) -> gpurun_out/prof5
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof5_bench.log 2>&1
