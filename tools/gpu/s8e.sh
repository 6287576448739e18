# round 6: ingress probe with K stagger, then K-staggered decode GEMMs (AKAP_GEMM_STAGGER=1)
# and the pgemm unit body with stagger: correctness under the flags, same-box A/B benches
set -u
O=gpurun_out/s8e; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
KG="decode_gemm or fused_decode_gemm or lds_dma_decode_gemm or kgemm or gemm_tuner or pgemm"
run ingress 300 ./tools/probes/ingress_probe "" 30 &&
AKAP_GEMM_STAGGER=1 AKAP_PGEMM_SCHED=3 AKAP_PGEMM_STAGGER=1 run t_stag 400 $P tests/test_kernels_gpu.py tests/test_fused_decode.py -k "$KG" &&
AKAP_PGEMM_SCHED=3 AKAP_PGEMM_STAGGER=1 run pg_s3stag 300 python -u tools/pgemm_bench.py --set verdict &&
run bench_s0 400 python -u bench.py &&
AKAP_GEMM_STAGGER=1 run bench_s1 400 python -u bench.py &&
run bench_s0b 400 python -u bench.py &&
AKAP_GEMM_STAGGER=1 run bench_s1b 400 python -u bench.py &&
run t_tpfault 300 $P tests/test_tp_gpu.py -k collective_timeout &&
echo done
