# round 6: unit-pipelined pgemm body (AKAP_PGEMM_SCHED=3) correctness + A/B vs hipBLASLt and
# the phase body; decode-GEMM ingress probe with XCD-mapping / operand modes + L2 hit counters
set -u
O=gpurun_out/s8b; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
K="pgemm_matches or pgemm_identity or pgemm_silu or pgemm_grouped"
AKAP_PGEMM_SCHED=3 run t_pg3 300 $P tests/test_kernels_gpu.py -k "$K" &&
run pg_sched1 300 python -u tools/pgemm_bench.py --set verdict &&
AKAP_PGEMM_SCHED=3 run pg_sched3 300 python -u tools/pgemm_bench.py --set verdict &&
run ingress 200 ./tools/probes/ingress_probe &&
run pmc_q00 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_q00 -o run -- ./tools/probes/ingress_probe "qkv,64x64,128,4,4,lds_counted,0,0" 5 &&
run pmc_q10 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_q10 -o run -- ./tools/probes/ingress_probe "qkv,64x64,128,4,4,lds_counted,1,0" 5 &&
run pmc_q01 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_q01 -o run -- ./tools/probes/ingress_probe "qkv,64x64,128,4,4,lds_counted,0,1" 5 &&
echo done
