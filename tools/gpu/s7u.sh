# prefill q prep with every operand load up front (one round trip), accumulators zeroed late:
# numerics, probe (plain vs qprep), engine tests, headline bench with kernel table
set -u
O=gpurun_out/s7u; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run t_attn 300 $P tests/test_kernels_gpu.py -k "prefill or attn or qk_norm or rope" &&
run t_engine 400 $P tests/test_engine_gpu.py &&
run t_tp 500 $P tests/test_tp_gpu.py &&
run t_pd 400 $P tests/test_pd_gpu.py &&
run attn 300 python -u tools/attn_prefill_probe.py --qprep &&
export AKAP_GEMM_TUNE_CACHE=/tmp/tune_qwen3.json &&
run tunecache 400 python -u bench.py --steps 1 --warmup 0 &&
run bench 400 python -u bench.py &&
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf -o run -- python3 bench.py --steps 1 --warmup 1 &&
python3 tools/prof_summary.py /tmp/pf/run_kernel_stats.csv > $O/kernel_stats.md && rm -rf /tmp/pf &&
echo done
