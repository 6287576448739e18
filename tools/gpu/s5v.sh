# pgemm early-issue schedule (AKAP_PGEMM_SCHED=2): numerics, prefill-shape A/B vs schedule 1 and
# hipBLASLt, split-K decode probe
set -u
O=gpurun_out/s5v; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
AKAP_PGEMM_SCHED=2 run t2 300 $P tests/test_kernels_gpu.py -k "pgemm" &&
AKAP_PGEMM_SCHED=2 run b2 400 python -u tools/pgemm_bench.py &&
run b1 400 python -u tools/pgemm_bench.py &&
AKAP_PGEMM_SCHED=2 run sk2 300 python -u tools/pgemm_m256_probe.py &&
echo done
