# round 3, batch 10: does warming the decode GEMM weights in MALL (AKAP_PREFETCH_WEIGHTS=1, an
# in-line prefetch kernel before each attention) shorten the fused GEMM chain?  kernel stats
# with and without; plus the graph-based CU-mask overlap probe
set -o pipefail
mkdir -p gpurun_out/pf
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 1 > gpurun_out/pf/warm.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pf/off -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/pf/off.log 2>&1 && \
AKAP_PREFETCH_WEIGHTS=1 AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pf/on -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/pf/on.log 2>&1 && \
timeout -k 10 300 python -u tools/cumask_probe.py > gpurun_out/cumask2.log 2>&1
