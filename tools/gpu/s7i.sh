# sampling: mixed-mode batches (new test) + the whole sampling/argmax test group
set -u
O=gpurun_out/s7i; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run t_samp 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sampl or argmax" &&
echo done
