# 8-wave prefill attention with a three-buffer K/V ring: numerics, timing, headline bench
set -u
O=gpurun_out/s7h; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run t_attn 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill or attn" &&
run attn 200 python -u tools/attn_prefill_probe.py &&
run bench1 400 python -u bench.py --steps 3 --warmup 1 &&
run bench2 400 python -u bench.py --steps 3 --warmup 1 &&
echo done
