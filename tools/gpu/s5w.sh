# EP=2 Qwen3-MoE rehearsal kernel table after the dispatch fixes (rank 0, torch.profiler)
set -u
O=gpurun_out/s5w; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
AKAP_MOE_MODE=ep run ep2_prof 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29623 bench.py --tp 2 --model qwen3-30b-a3b --dist-backend gloo --gpus 1 --steps 1 --warmup 1 --output-len 8 --torch-profile &&
echo done
