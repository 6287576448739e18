# round 6: 256x256 LM-head form (AKAP_WGEMM_WIDE=1): correctness, LM-head probe A/B, headline A/B
set -u
O=gpurun_out/s8g; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
AKAP_WGEMM_WIDE=1 run t_wide 300 $P tests/test_kernels_gpu.py -k "wide_row_gemm" &&
run lm_w0 200 python -u tools/lmhead_probe.py &&
AKAP_WGEMM_WIDE=1 run lm_w1 200 python -u tools/lmhead_probe.py &&
run bench_w0 400 python -u bench.py &&
AKAP_WGEMM_WIDE=1 run bench_w1 400 python -u bench.py &&
run bench_w0b 400 python -u bench.py &&
AKAP_WGEMM_WIDE=1 run bench_w1b 400 python -u bench.py &&
echo done
