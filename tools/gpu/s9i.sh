# round 6: tuner timed on a cold-sized layer subset: Llama-3-8B cold tuning time + tok/s,
# Qwen3 headline regression check, fused-chain GPU tests
set -u
O=gpurun_out/s9i; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run t_fused 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_decode.py &&
AKAP_GEMM_TUNE_VERBOSE=1 run llama8b 900 python -u bench.py --model llama-3-8b &&
run qwen 400 python -u bench.py &&
echo done
