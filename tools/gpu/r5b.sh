set -u
O=gpurun_out/r5c; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
run t 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k h2d &&
run te 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_tp_gpu.py tests/test_pd_gpu.py &&
run bench 600 python -u bench.py &&
AKAP_H2D_KERNEL=0 run bench_memcpy 600 python -u bench.py &&
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5cprof -o run -- python3 bench.py --steps 2 --warmup 1 &&
run gaps 120 python -u bench/step_gaps.py /tmp/r5cprof/run_kernel_trace.csv
rm -rf /tmp/r5cprof
echo done
