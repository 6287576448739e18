# LM head at decode batch sizes: hipBLASLt / wgemm / gdgemm 256-row / pgemm on a 256-padded table
set -u
O=gpurun_out/s6l; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run lm 300 python -u tools/lmhead_probe.py &&
echo done
