# headline bench repeated 3x on the final tree (variance band) + fp8-KV variant refresh
set -u
O=gpurun_out/r5j; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run b1 600 python -u bench.py &&
run b2 600 python -u bench.py &&
run b3 600 python -u bench.py &&
run fp8kv 600 python -u bench.py --kv-cache-dtype fp8 &&
echo done
