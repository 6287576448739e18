# EP=2 Qwen3-MoE rehearsal with the IPC row-slab all-gather; two-pod P/D GPU test, server-load metrics (default T=1.0 requests), kernel table at T=1.0
set -u
O=gpurun_out/s5f; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -v --timeout 400 --timeout-method thread"
AKAP_MOE_MODE=ep run ep2_qwen3moe 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29623 bench.py --tp 2 --model qwen3-30b-a3b --dist-backend gloo --gpus 1 --steps 2 --warmup 1 &&
run pd_gpu 600 $P tests/test_pd_gpu.py &&
run metrics 300 python -u tools/metrics_load_probe.py --out $O/metrics &&
run prof_t1 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t1 -o run -- python3 bench.py --temperature 1.0 --steps 1 --warmup 1 &&
echo done
