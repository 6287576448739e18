# H2D fallback probe check: engine GPU tests, smoke, one bench
set -u
O=gpurun_out/r5h; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run engine 600 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
run bench 600 python -u bench.py &&
echo done
