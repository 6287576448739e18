# fp8-cache prefill with the q prep: kernel test + fp8 KV bench (regression check)
set -u
O=gpurun_out/s7o; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run t_q 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "qprep" &&
run fp8 400 python -u bench.py --kv-cache-dtype fp8 &&
echo done
