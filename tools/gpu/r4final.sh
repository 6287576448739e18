# round-4 checkpoint (profile summarised on the box, raw traces deleted: gpurun_out <= 64 MiB)
set -u
O=gpurun_out/r5d; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
run suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
run bench 600 python -u bench.py &&
run bench2 600 python -u bench.py &&
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5dprof -o run -- python3 bench.py --steps 2 --warmup 1 &&
cp /tmp/r5dprof/run_kernel_stats.csv $O/kernel_stats.csv &&
run gaps 120 python -u bench/step_gaps.py /tmp/r5dprof/run_kernel_trace.csv &&
rm -rf /tmp/r5dprof
echo done
echo done
