# clean steady-state kernel table of the final round-5 tree (GEMM plan from the tuning cache,
# no tuner launches), greedy and T = 1.0; headline bench for the same box
set -u
O=gpurun_out/s7s; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
export AKAP_GEMM_TUNE_CACHE=/tmp/tune_qwen3.json
run tunecache 400 python -u bench.py --steps 1 --warmup 0 &&
run bench 400 python -u bench.py &&
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf -o run -- python3 bench.py --steps 1 --warmup 1 &&
python3 tools/prof_summary.py /tmp/pf/run_kernel_stats.csv > $O/kernel_stats.md && rm -rf /tmp/pf &&
echo done
