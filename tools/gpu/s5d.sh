# EP prefill on the fixed-capacity dispatch (Qwen3-30B-A3B EP=2, two ranks on one GPU); TP=4 at
# Llama-3-70B widths (test + bench); two-pod P/D http bootstrap; sampler at T=1.0 in the bench
# (with a kernel table); moe expert rows with empty slots
set -u
O=gpurun_out/s5d; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -v --timeout 400 --timeout-method thread"
run moe_rows 300 $P tests/test_kernels_gpu.py -k "expert_rows or moe_block" &&
run tp4_70b 500 $P tests/test_tp_gpu.py -k "tp4_llama70b" &&
run tp_all 600 $P tests/test_tp_gpu.py -k "ep" &&
AKAP_MOE_MODE=ep run ep2_qwen3moe 700 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29623 bench.py --tp 2 --model qwen3-30b-a3b --dist-backend gloo --gpus 1 --steps 2 --warmup 1 &&
run tp4_70b_bench 700 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29624 bench.py --tp 4 --model llama-3-70b-l4 --dist-backend gloo --gpus 1 --steps 2 --warmup 1 &&
run pd_gpu 600 $P tests/test_pd_gpu.py &&
run metrics 300 python -u tools/metrics_load_probe.py --out $O/metrics &&
run bench_t1 400 python -u bench.py --temperature 1.0 &&
run prof_t1 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t1 -o run -- python3 bench.py --temperature 1.0 --steps 1 --warmup 1 &&
echo done
