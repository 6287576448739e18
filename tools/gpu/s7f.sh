# regression checks on the final tree: fp8 KV bench, TP=2 Qwen3 (two ranks on one GPU), P/D Qwen3 1P:1D
set -u
O=gpurun_out/s7f; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
TR="python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631"
run fp8 400 python -u bench.py --kv-cache-dtype fp8 &&
run tp2_qwen 600 $TR bench.py --tp 2 --dist-backend gloo --gpus 1 &&
run pd_qwen 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29632 bench.py --mode pd --dist-backend gloo --kv-transport ipc --gpus 1 --steps 2 &&
echo done
