# P/D over the hipIpc pull on one MI355X (two ranks share the device), Llama-3-8B headline
# P/D config + Qwen3 quick check; then the full GPU suite and smoke
set -u
O=gpurun_out/r4b; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
TR="python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611"
run pd_qwen 420 $TR bench.py --mode pd --dist-backend gloo --kv-transport ipc --gpus 1 &&
run pd_llama 900 $TR bench.py --mode pd --model llama-3-8b --dist-backend gloo --kv-transport ipc --gpus 1 &&
echo done
run rehearsal70b 600 python -u bench/tp_shard_rehearsal.py --B 64,256 &&
echo done2
