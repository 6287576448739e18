# pipelined 8-wave prefill attention (AKAP_ATTN_PIPE=1): numerics, timing A/B, headline bench A/B
set -u
O=gpurun_out/s7k; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
AKAP_ATTN_PIPE=1 run t_attn 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill or attn" &&
run attn0 200 python -u tools/attn_prefill_probe.py --rows 256 &&
AKAP_ATTN_PIPE=1 run attn1 200 python -u tools/attn_prefill_probe.py --rows 256 &&
AKAP_ATTN_PIPE=1 run bench1 400 python -u bench.py --steps 3 --warmup 1 &&
run bench0 400 python -u bench.py --steps 3 --warmup 1 &&
echo done
