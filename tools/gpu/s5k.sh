# K13 grid per communicator (ranks sharing a GPU: 128 / world blocks): custom-collective tests,
# TP/EP process tests, TP=4 70B-width bench; 1P:2D P/D with 30 GiB caches (one export
# allocation each) on the ipc transport
set -u
O=gpurun_out/s5k; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run car 300 $P tests/test_custom_allreduce_gpu.py &&
run tp 500 $P tests/test_tp_gpu.py &&
run pd1p2d 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --mode pd --pd-prefill-ranks 1 --dist-backend gloo --steps 2 --num-gpu-blocks 8192 &&
run tp4_70b_bench 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29624 bench.py --tp 4 --model llama-3-70b-l4 --dist-backend gloo --gpus 1 --steps 1 --warmup 1 --input-len 512 --output-len 64 --max-num-batched-tokens 512 &&
echo done
