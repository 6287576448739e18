# round 6: decode down projection with the split-K combine inside the launch (dgemm SPL 2):
# correctness, then same-box A/B of the headline with / without the new candidates
set -u
O=gpurun_out/s9a; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run t_inl 400 $P tests/test_kernels_gpu.py tests/test_fused_decode.py -k "register_ring_inlaunch or decode_gemm or fused" &&
AKAP_GEMM_TUNE_VERBOSE=1 run bench_i1 400 python -u bench.py &&
AKAP_GEMM_TUNE_VERBOSE=1 AKAP_DGEMM_RR_INL=0 run bench_i0 400 python -u bench.py &&
AKAP_GEMM_TUNE_VERBOSE=1 run bench_i1b 400 python -u bench.py &&
AKAP_GEMM_TUNE_VERBOSE=1 AKAP_DGEMM_RR_INL=0 run bench_i0b 400 python -u bench.py &&
echo done
