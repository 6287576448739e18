# round 6: V span role with every read issued up front (rope_cache.hip): rope/cache/tail tests,
# the rope probe (serving form), a serving kernel trace
set -u
O=gpurun_out/s9y; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run t_rope 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py -k "rope or tail or cache or prefill" &&
run t_engine 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py &&
run rope 300 python -u tools/rope_probe.py &&
run prof 600 rocprofv3 --kernel-trace --stats -d /tmp/p1 -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 1 &&
run prof_s 120 python3 tools/prof_summary.py /tmp/p1/run_kernel_trace.csv $O/prof.md "V span preload" &&
run b1 400 python -u bench.py &&
echo done
