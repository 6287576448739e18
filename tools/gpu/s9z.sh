# round 6, tree check: every GPU test file, smoke, headline bench x2 (+ T = 1.0), a serving
# kernel trace of the bench, Llama-3-8B (cold tuning time), then the 1P:2D hipIpc sweep LAST
# (it stops the script at its first hang).  Traces stay in /tmp on the box (gpurun_out <= 64 MiB)
set -u
O=gpurun_out/s9z; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
run t_kernels 900 $P tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py tests/test_fused_decode.py &&
run t_car 300 $P tests/test_custom_allreduce_gpu.py &&
run t_tp 500 $P tests/test_tp_gpu.py &&
run t_pd 400 $P tests/test_pd_gpu.py &&
run t_engine 500 $P tests/test_engine_gpu.py &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
run bench_a 400 python -u bench.py &&
run bench_b 400 python -u bench.py &&
run bench_t1 400 python -u bench.py --temperature 1.0 &&
run prof 600 rocprofv3 --kernel-trace --stats -d /tmp/s9zprof -o run --output-format csv -- python3 -u bench.py --steps 2 --warmup 1 &&
run prof_serving 120 python3 tools/prof_summary.py /tmp/s9zprof/run_kernel_trace.csv $O/prof_serving.md "Qwen3-0.6B headline bench, serving dispatches only" &&
run prof_gaps 120 python3 tools/trace_gaps.py /tmp/s9zprof/run_kernel_trace.csv &&
cp /tmp/s9zprof/run_kernel_stats.csv $O/prof_kernel_stats.csv &&
run llama8b 900 python -u bench.py --model llama-3-8b &&
run ipc2 600 bash tools/gpu/s9_ipc_sweep2.sh &&
echo done
