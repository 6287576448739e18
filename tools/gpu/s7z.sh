# last sanity on the final build: qprep/attention kernel tests, engine tests, smoke, bench
set -u
O=gpurun_out/s7z; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run t_k 300 $P tests/test_kernels_gpu.py -k "qprep or prefill or sampl" &&
run t_engine 400 $P tests/test_engine_gpu.py &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
run bench 400 python -u bench.py &&
echo done
