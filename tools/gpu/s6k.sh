# sampler rework II in the engine: engine tests, bench at T=1.0, headline bench, kernel table at T=1.0
set -u
O=gpurun_out/s6k; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
run t_kernels 900 $P tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py &&
run t_engine 400 $P tests/test_engine_gpu.py &&
run bench_t1 400 python -u bench.py --temperature 1.0 &&
run bench 400 python -u bench.py &&
run prof_t1 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf -o run -- python3 bench.py --temperature 1.0 --steps 1 --warmup 1 &&
python3 tools/prof_summary.py /tmp/pf/run_kernel_stats.csv > $O/kernel_stats_t1.md && rm -rf /tmp/pf &&
echo done
