# (re-run of s5f, whose 64+ MiB rocprof directory kept every log from coming back) EP=2 Qwen3-MoE
# rehearsal; two-pod P/D GPU test; server-load metrics window (default T=1.0 requests); kernel
# table of the T=1.0 bench (summary only; the raw trace stays in /tmp)
set -u
O=gpurun_out/s5i; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -v --timeout 400 --timeout-method thread"
AKAP_MOE_MODE=ep run ep2_qwen3moe 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29623 bench.py --tp 2 --model qwen3-30b-a3b --dist-backend gloo --gpus 1 --steps 2 --warmup 1 &&
run pd_gpu 600 $P tests/test_pd_gpu.py &&
run metrics 300 python -u tools/metrics_load_probe.py --out $O/metrics &&
run bench_t1 400 python -u bench.py --temperature 1.0 &&
run prof_t1 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt1 -o run -- python3 bench.py --temperature 1.0 --steps 1 --warmup 1 &&
python3 tools/prof_summary.py /tmp/pt1/run_kernel_stats.csv > $O/t1_kernel_stats.md && rm -rf /tmp/pt1 &&
echo done
