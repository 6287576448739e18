# round 6: prefill attention with the deferred running max (AKAP_FA_RESCALE_T, default 8) vs the
# exact max (0): attention tests, micro (128- and 256-row tiles), headline A/B
set -u
O=gpurun_out/s9p; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run t_attn 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or prefill" &&
run ap8 300 python -u tools/attn_prefill_probe.py &&
AKAP_FA_RESCALE_T=0 run ap0 300 python -u tools/attn_prefill_probe.py &&
run b8a 400 python -u bench.py &&
AKAP_FA_RESCALE_T=0 run b0a 400 python -u bench.py &&
run b8b 400 python -u bench.py &&
AKAP_FA_RESCALE_T=0 run b0b 400 python -u bench.py &&
echo done
