# round 6: fused decode attention with the new token's K/V stores deferred to the end of the
# work item (AKAP_DECODE_DEFER_KV, default 1): decode/tail tests, attention A/B, headline A/B
set -u
O=gpurun_out/s9zf; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run t_dec 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_decode.py tests/test_kernels_gpu.py -k "decode or tail or fused" &&
run ab1 300 python -u bench/attn_fused_ab.py &&
AKAP_DECODE_DEFER_KV=0 run ab0 300 python -u bench/attn_fused_ab.py &&
run t_engine 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py &&
run b1a 400 python -u bench.py &&
AKAP_DECODE_DEFER_KV=0 run b0a 400 python -u bench.py &&
run b1b 400 python -u bench.py &&
AKAP_DECODE_DEFER_KV=0 run b0b 400 python -u bench.py &&
echo done
