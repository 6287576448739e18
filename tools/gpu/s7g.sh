# ring GEMM experiment (loader / consumer waves) vs hipBLASLt at M = 256
set -u
O=gpurun_out/s7g; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run rg 120 python -u tools/rgemm_probe.py &&
echo done
