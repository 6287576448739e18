# round 6, final verification after the decode launch-bounds change: kernel + engine tests, smoke,
# headline x2, Llama-3-8B
set -u
O=gpurun_out/s9zr; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run t_kernels 900 $P tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py tests/test_fused_decode.py &&
run t_rest 900 $P tests/test_engine_gpu.py tests/test_pd_gpu.py tests/test_tp_gpu.py tests/test_custom_allreduce_gpu.py &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
run bench_a 400 python -u bench.py &&
run bench_b 400 python -u bench.py &&
run llama8b 900 python -u bench.py --model llama-3-8b &&
echo done
