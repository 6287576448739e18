# Burst headline with mixed batching on / off (same build, back to back)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
set -e
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > gpurun_out/r2_burst_mixed.log 2>&1
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-mixed-batching > gpurun_out/r2_burst_pfirst.log 2>&1
echo ab ok
