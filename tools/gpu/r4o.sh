set -u
O=gpurun_out/r4o; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
run moeprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/moep -o run -- python3 bench.py --model qwen3-30b-a3b --steps 1 --warmup 0 &&
python3 tools/prof_summary.py /tmp/moep/run_kernel_stats.csv > $O/moe_kernel_stats.md && rm -rf /tmp/moep &&
export AKAP_GEMM_TUNE_CACHE=/tmp/tune_qwen3.json &&
run tunecache 300 python3 bench.py --steps 1 --warmup 0 &&
run qprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/qp -o run -- python3 bench.py --steps 2 --warmup 1 &&
python3 tools/prof_summary.py /tmp/qp/run_kernel_stats.csv > $O/qwen3_kernel_stats.md &&
python3 bench/step_gaps.py /tmp/qp/run_kernel_trace.csv > $O/qwen3_gaps.log; rm -rf /tmp/qp
echo done
