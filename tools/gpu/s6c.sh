# Llama-3-8B P/D 1P:1D on one GPU with the 28 GiB shared-GPU cache cap (ipc transport)
set -u
O=gpurun_out/s6c; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run pd_llama8b 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --mode pd --model llama-3-8b --dist-backend gloo --kv-transport ipc --gpus 1 --steps 2 &&
echo done
