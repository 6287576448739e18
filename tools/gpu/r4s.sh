set -u
O=gpurun_out/r4s; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
run tk 300 $P tests/test_kernels_gpu.py -k "pgemm or moe or router" &&
run te 300 $P tests/test_engine_gpu.py -k "moe or mixtral or hand_written" &&
run bench 600 python -u bench.py
echo done
