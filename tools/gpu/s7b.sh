# final round-5 tree check: every GPU test file, smoke, headline bench x2, T=1.0 bench, clean kernel table
set -u
O=gpurun_out/s7b; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
run t_kernels 900 $P tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py &&
run t_car 300 $P tests/test_custom_allreduce_gpu.py &&
run t_tp 500 $P tests/test_tp_gpu.py &&
run t_pd 400 $P tests/test_pd_gpu.py &&
run t_engine 400 $P tests/test_engine_gpu.py &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
run bench 400 python -u bench.py &&
run bench_b 400 python -u bench.py &&
run bench_t1 400 python -u bench.py --temperature 1.0 &&
export AKAP_GEMM_TUNE_CACHE=/tmp/tune_qwen3.json &&
run tunecache 400 python -u bench.py --steps 1 --warmup 0 &&
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf -o run -- python3 bench.py --steps 1 --warmup 1 &&
python3 tools/prof_summary.py /tmp/pf/run_kernel_stats.csv > $O/kernel_stats.md && rm -rf /tmp/pf &&
run prof_t1 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf1 -o run -- python3 bench.py --steps 1 --warmup 1 --temperature 1.0 &&
python3 tools/prof_summary.py /tmp/pf1/run_kernel_stats.csv > $O/kernel_stats_t1.md && rm -rf /tmp/pf1 &&
echo done
