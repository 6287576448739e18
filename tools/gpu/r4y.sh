set -u
O=gpurun_out/r4z; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run car 300 $P tests/test_custom_allreduce_gpu.py -k "alltoall" &&
run tpt 500 $P tests/test_tp_gpu.py &&
AKAP_MOE_MODE=ep AKAP_BENCH_STACKS=100 run ep2_qwen3moe 700 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29623 bench.py --tp 2 --model qwen3-30b-a3b --dist-backend gloo --gpus 1
echo done
