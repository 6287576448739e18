# kCarU=8: IPC collective tests + EP=2 Qwen3-MoE rehearsal (prefill time after the unroll)
set -u
O=gpurun_out/s5z; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_custom_allreduce_gpu.py &&
AKAP_MOE_MODE=ep run ep2 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29624 bench.py --tp 2 --model qwen3-30b-a3b --dist-backend gloo --gpus 1 --steps 1 --warmup 1 --output-len 8 &&
echo done
