# prefill attention: static priority for the second half of the waves (AKAP_ATTN_PRIO=1), A/B
set -u
O=gpurun_out/s7r; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
AKAP_ATTN_PRIO=1 run t_attn 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill" &&
run a0 200 python -u tools/attn_prefill_probe.py &&
AKAP_ATTN_PRIO=1 run a1 200 python -u tools/attn_prefill_probe.py &&
run a0b 200 python -u tools/attn_prefill_probe.py &&
AKAP_ATTN_PRIO=1 run a1b 200 python -u tools/attn_prefill_probe.py &&
echo done
