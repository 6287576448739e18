# GPU verification of the current tree: gpu tests, smoke, headline bench, kernel stats.
# usage: gpurun --timeout 1100 -- 'bash bench/gpu_verify.sh TAG'
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
TAG=${1:-verify}
set -e
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
echo "gpu tests ok"
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
echo "smoke ok"
# the bench run tunes and saves the GEMM plan; the profiled run reloads it, so its kernel
# stats hold the serving kernels only (no tuning candidates)
export AKAP_GEMM_TUNE_CACHE=gpurun_out/${TAG}_tune.json
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 > gpurun_out/${TAG}_bench.log 2>&1
echo "bench ok"
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/${TAG}_prof.log 2>&1
echo "prof ok"
# keep only the stats summaries (the full trace would exceed gpurun's 64 MiB pull-back)
find gpurun_out/${TAG}_prof -type f ! -name '*stats*' -delete
