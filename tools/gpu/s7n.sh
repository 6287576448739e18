# model refreshes after the prefill q-prep fusion (TTFT): Llama-3-8B, Qwen3 16k context, Mixtral,
# Llama-3-8B P/D on one GPU
set -u
O=gpurun_out/s7n; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run llama8b 600 python -u bench.py --model llama-3-8b --steps 2 &&
run longctx 400 python -u bench.py --num-requests 64 --input-len 16384 --max-model-len 20480 --steps 1 &&
run mixtral 600 python -u bench.py --model mixtral-8x7b --num-requests 128 --max-num-seqs 128 --steps 1 &&
echo done
