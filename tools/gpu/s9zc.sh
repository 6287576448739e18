# round 6: bulk admission with int32 prompt arrays (one copy per request into the scheduler,
# params normalized once per batch): engine tests, headline x2, prefill-phase trace
set -u
O=gpurun_out/s9zc; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run t_engine 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py &&
run b1 400 python -u bench.py &&
run b2 400 python -u bench.py &&
run prof 600 rocprofv3 --kernel-trace -d /tmp/pp -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 1 &&
run phase 120 python3 tools/prefill_phase.py /tmp/pp/run_kernel_trace.csv &&
echo done
