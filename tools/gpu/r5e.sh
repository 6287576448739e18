set -u
O=gpurun_out/r5e; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
AKAP_PGEMM_GM=4 run gm4 300 python -u tools/pgemm_bench.py &&
run gm8 300 python -u tools/pgemm_bench.py &&
AKAP_PGEMM_GM=16 run gm16 300 python -u tools/pgemm_bench.py &&
AKAP_PGEMM_GM=32 run gm32 300 python -u tools/pgemm_bench.py
echo done
