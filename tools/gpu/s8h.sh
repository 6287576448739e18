# round 6: prefill-attention compute/load ping-pong (AKAP_PREFILL_STAGGER=1): correctness,
# kernel A/B at the verdict shapes, headline A/B
set -u
O=gpurun_out/s8h; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
AKAP_PREFILL_STAGGER=1 run t_pstag 300 $P tests/test_kernels_gpu.py -k "paged_attention_prefill" &&
run ap_s0 200 python -u tools/attn_prefill_probe.py --rows 256 &&
AKAP_PREFILL_STAGGER=1 run ap_s1 200 python -u tools/attn_prefill_probe.py --rows 256 &&
run bench_p0 400 python -u bench.py &&
AKAP_PREFILL_STAGGER=1 run bench_p1 400 python -u bench.py &&
run bench_p0b 400 python -u bench.py &&
AKAP_PREFILL_STAGGER=1 run bench_p1b 400 python -u bench.py &&
echo done
