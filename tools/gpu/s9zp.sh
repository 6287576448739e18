# round 6 late: prefill chunk budget (max_num_batched_tokens) vs headline tok/s and p50 TTFT
set -u
O=gpurun_out/s9zp; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc $(grep -o '"value": [0-9.]*\|"p50_ttft_ms": [0-9.]*' $O/$n.log | tr '\n' ' ')"; [ $rc -eq 0 ]; }
run c16k_a 400 python -u bench.py &&
run c8k_a 400 python -u bench.py --max-num-batched-tokens 8192 &&
run c12k_a 400 python -u bench.py --max-num-batched-tokens 12288 &&
run c16k_b 400 python -u bench.py &&
run c8k_b 400 python -u bench.py --max-num-batched-tokens 8192 &&
run c12k_b 400 python -u bench.py --max-num-batched-tokens 12288 &&
echo done
