# EP=2 Qwen3-MoE rehearsal at the s5d config (steps 2, warmup 1) after the chunked dispatch + unrolled IPC a2a
set -u
O=gpurun_out/s6a; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
AKAP_MOE_MODE=ep run ep2_qwen3moe 700 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29623 bench.py --tp 2 --model qwen3-30b-a3b --dist-backend gloo --gpus 1 --steps 2 --warmup 1 &&
echo done
