# Mixtral repeat (TTFT noise check)
set -u
O=gpurun_out/s7d; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run mixtral 900 python -u bench.py --model mixtral-8x7b --num-requests 128 --max-num-seqs 128 --steps 2 &&
echo done
