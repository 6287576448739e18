# per-step prefill tile rows (256-row kernel for short chunks): engine tests + headline bench
set -u
O=gpurun_out/s6v; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
run t_engine 400 $P tests/test_engine_gpu.py tests/test_tp_gpu.py &&
run bench 400 python -u bench.py &&
AKAP_PREFILL_TILE_ROWS=128 run bench128 400 python -u bench.py &&
echo done
