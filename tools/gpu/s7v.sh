# final round-5 tree check: every GPU test file, smoke, headline bench x2, T=1.0
set -u
O=gpurun_out/s7v; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
run t_kernels 900 $P tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py &&
run t_car 300 $P tests/test_custom_allreduce_gpu.py &&
run t_tp 500 $P tests/test_tp_gpu.py &&
run t_pd 400 $P tests/test_pd_gpu.py &&
run t_engine 400 $P tests/test_engine_gpu.py &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
run bench 400 python -u bench.py &&
run bench_b 400 python -u bench.py &&
run bench_t1 400 python -u bench.py --temperature 1.0 &&
echo done
