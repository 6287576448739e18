# round 6 late: model refresh after the longest-first prefill grid -- long context (Qwen3 16k,
# Llama-3-8B 7k) and the MoE models
set -u
O=gpurun_out/s9zi; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run qwen16k 600 python -u bench.py --num-requests 64 --max-num-seqs 64 --input-len 16384 --max-model-len 20480 --steps 1 &&
run llama7k 600 python -u bench.py --model llama-3-8b --num-requests 32 --max-num-seqs 32 --input-len 7000 --output-len 128 --max-model-len 8192 --steps 1 &&
run mixtral 600 python -u bench.py --model mixtral-8x7b --num-requests 128 --max-num-seqs 128 --steps 1 &&
run qwen3moe 600 python -u bench.py --model qwen3-30b-a3b --steps 2 &&
echo done
