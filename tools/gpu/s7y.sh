# qk_norm_rope_cache: first head-row batch requested before the rotary chain -- numerics,
# engine, TP/PD, kernel table with the tuning cache, headline bench
set -u
O=gpurun_out/s7y; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run t_k 300 $P tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py -k "rope or qk_norm or prefill or attn or cache" &&
run t_engine 400 $P tests/test_engine_gpu.py &&
run t_tp 500 $P tests/test_tp_gpu.py &&
run t_pd 400 $P tests/test_pd_gpu.py &&
export AKAP_GEMM_TUNE_CACHE=/tmp/tune_qwen3.json &&
run tunecache 400 python -u bench.py --steps 1 --warmup 0 &&
run bench 400 python -u bench.py &&
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf -o run -- python3 bench.py --steps 1 --warmup 1 &&
python3 tools/prof_summary.py /tmp/pf/run_kernel_stats.csv > $O/kernel_stats.md && rm -rf /tmp/pf &&
echo done
