set -u
O=gpurun_out/r5f; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
run lc_qwen 600 python -u bench.py --num-requests 64 --max-num-seqs 64 --input-len 16384 --output-len 256 --max-model-len 20480 --steps 1 &&
run lc_llama 600 python -u bench.py --model llama-3-8b --num-requests 32 --max-num-seqs 32 --input-len 7000 --output-len 128 --max-model-len 8192 --steps 1
echo done
