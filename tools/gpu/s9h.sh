# round 6: P/D on the hipIpc pull WITHOUT the 28 GiB cache cap (KV segments sized around the
# runtime's bit-31 hipIpcOpenMemHandle hang): 1P:1D Llama-3-8B and 1P:2D Qwen3 on one GPU
set -u
O=gpurun_out/s9h; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
TR="python -u -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run t_pd 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pd_gpu.py &&
run pd_llama 900 $TR --nproc-per-node 2 --master-port 29611 bench.py --mode pd --model llama-3-8b --dist-backend gloo --kv-transport ipc --gpus 1 &&
run pd1p2d 600 $TR --nproc-per-node 3 --master-port 29517 bench.py --gpus 1 --mode pd --pd-prefill-ranks 1 --dist-backend gloo --kv-transport ipc --steps 2 &&
echo done
