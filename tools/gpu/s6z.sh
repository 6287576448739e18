# greedy decode: LM head fused with the argmax (no logits); tests + bench A/B
set -u
O=gpurun_out/s6z; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
run t_k 300 $P tests/test_kernels_gpu.py -k "lm_head or argmax or wgemm" &&
run t_engine 400 $P tests/test_engine_gpu.py tests/test_tp_gpu.py &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
run bench 400 python -u bench.py &&
AKAP_LM_ARGMAX=0 run bench_off 400 python -u bench.py &&
run bench_b 400 python -u bench.py &&
echo done
