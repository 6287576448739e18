# sampler passes v3b + greedy argmax graph variant: tests, microbench, headline bench (greedy) and
# T=1.0; EP rehearsal kernel table (s5l's ep2_prof log kept)
set -u
O=gpurun_out/s5m; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run samp_t 300 $P tests/test_kernels_gpu.py -k "sampl or argmax" &&
run samp_b 300 python -u tools/sample_bench.py &&
run engine_t 600 $P tests/test_engine_gpu.py &&
run bench 400 python -u bench.py &&
run bench_t1 400 python -u bench.py --temperature 1.0 &&
echo done
