# model refreshes on the final round-5 tree: Llama-3-8B, Qwen3-30B-A3B, Mixtral-8x7B, Qwen3 long context
set -u
O=gpurun_out/s7c; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run llama8b 900 python -u bench.py --model llama-3-8b --steps 2 &&
run qwen3moe 900 python -u bench.py --model qwen3-30b-a3b --steps 2 &&
run mixtral 900 python -u bench.py --model mixtral-8x7b --num-requests 128 --max-num-seqs 128 --steps 1 &&
run longctx 900 python -u bench.py --num-requests 64 --input-len 16384 --max-model-len 20480 --steps 1 &&
echo done
