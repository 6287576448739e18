# production multi-rank decode paths at real model sizes, two ranks sharing one MI355X (gloo
# control plane; collectives = the custom IPC kernels inside the captured decode graphs)
set -u
O=gpurun_out/r4w; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
TR="python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621"
run tpt 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tp_gpu.py tests/test_custom_allreduce_gpu.py &&
AKAP_BENCH_STACKS=100 run tp2_qwen 500 $TR bench.py --tp 2 --dist-backend gloo --gpus 1 &&
AKAP_BENCH_STACKS=100 run tp2_llama8b 700 $TR bench.py --tp 2 --model llama-3-8b --dist-backend gloo --gpus 1
echo done
