# LM head: wgemm + argmax vs the fused ARGMAX epilogue
set -u
O=gpurun_out/s7a; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run lm 300 python -u tools/lmhead_probe.py &&
echo done
