# round 6: prefill tile policy flipped (256 rows default, 128 for short prompts): engine tests,
# headline x2, Llama-3-8B headline
set -u
O=gpurun_out/s9z; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run t_engine 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py &&
run b1 400 python -u bench.py &&
run b2 400 python -u bench.py &&
run llama 900 python -u bench.py --model llama-3-8b &&
echo done
