# 70B TP=8 rank rehearsal refresh; Mixtral repeat (TTFT variance check)
set -u
O=gpurun_out/s5u; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run rehearsal70b 600 python -u bench/tp_shard_rehearsal.py --B 64,256 &&
run mixtral 900 python -u bench.py --model mixtral-8x7b --num-requests 128 --steps 2 &&
echo done
