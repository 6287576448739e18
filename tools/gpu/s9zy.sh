# round 6, closing tree check (late tree + scalar q-norm weight loads in prefill q prep):
# every GPU test file, smoke, headline x2 + T=1, serving kernel trace + decode boundaries,
# Llama-3-8B, P/D ipc, the self-launched 2-rank bench (ranks sharing the GPU over gloo)
set -u
O=gpurun_out/s9zy; mkdir -p $O
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
run prof 600 rocprofv3 --kernel-trace --stats -d /tmp/s9zyprof -o run --output-format csv -- python3 -u bench.py --steps 2 --warmup 1 &&
run prof_serving 120 python3 tools/prof_summary.py /tmp/s9zyprof/run_kernel_trace.csv $O/prof_serving.md "Qwen3-0.6B headline bench, serving dispatches only" &&
run prof_gaps 120 python3 tools/trace_gaps.py /tmp/s9zyprof/run_kernel_trace.csv &&
run prof_bounds 120 python3 tools/decode_boundaries.py /tmp/s9zyprof/run_kernel_trace.csv &&
cp /tmp/s9zyprof/run_kernel_stats.csv $O/prof_kernel_stats.csv &&
run llama8b 900 python -u bench.py --model llama-3-8b &&
run pd_llama 900 python -u -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 2 --master-port 29611 bench.py --mode pd --model llama-3-8b --dist-backend gloo --kv-transport ipc --gpus 1 &&
run gpus2_gloo 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 1 --warmup 1 &&
echo done
