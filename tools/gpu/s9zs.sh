# round 6 final: long-context and fp8-KV regression check after the decode launch-bounds change
set -u
O=gpurun_out/s9zs; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc $(grep -o '"value": [0-9.]*\|"p50_ttft_ms": [0-9.]*' $O/$n.log | tr '\n' ' ')"; [ $rc -eq 0 ]; }
run qwen16k 600 python -u bench.py --num-requests 64 --max-num-seqs 64 --input-len 16384 --max-model-len 20480 --steps 1 &&
run fp8kv 400 python -u bench.py --kv-cache-dtype fp8 &&
echo done
