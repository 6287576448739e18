# P/D rehearsals with the 28 GiB cache cap (Llama-3-8B 1P:1D over ipc; Qwen3 1P:2D); Mixtral
# refresh; sampler tests on the restored per-lane passes
set -u
O=gpurun_out/s5t; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run samp_t 300 $P tests/test_kernels_gpu.py -k "sampl or argmax" &&
run pd1p2d 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --mode pd --pd-prefill-ranks 1 --dist-backend gloo --steps 2 &&
run pd_llama8b 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --mode pd --model llama-3-8b --dist-backend gloo --kv-transport ipc --gpus 1 --steps 2 &&
run mixtral 900 python -u bench.py --model mixtral-8x7b --num-requests 128 --steps 2 &&
echo done
