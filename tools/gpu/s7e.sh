# final .so (comment-only sampler change): kernel tests, smoke, bench
set -u
O=gpurun_out/s7e; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
run t_kernels 900 $P tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py &&
run t_engine 400 $P tests/test_engine_gpu.py &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
run bench 400 python -u bench.py &&
echo done
