set -u
O=gpurun_out/r5g; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
run q_mixed 400 python -u bench.py &&
run q_pf 400 python -u bench.py --no-mixed-batching &&
run l_mixed 600 python -u bench.py --model llama-3-8b --steps 2 &&
run l_pf 600 python -u bench.py --model llama-3-8b --steps 2 --no-mixed-batching
echo done
