# round 6: L2 hit rate of the prefill GEMMs, hipBLASLt vs pgemm (8-wave and unit body)
set -u
O=gpurun_out/s8f; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run l2_s1 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/l2_s1 -o run -- python3 tools/gemm_l2_probe.py &&
AKAP_PGEMM_SCHED=3 run l2_s3 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/l2_s3 -o run -- python3 tools/gemm_l2_probe.py &&
run l2_t1 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/l2_t1 -o run -- python3 tools/gemm_l2_probe.py &&
AKAP_PGEMM_GM=4 run pg_gm4 300 python -u tools/pgemm_bench.py --set verdict &&
AKAP_PGEMM_GM=2 run pg_gm2 300 python -u tools/pgemm_bench.py --set verdict &&
AKAP_PGEMM_GM=16 run pg_gm16 300 python -u tools/pgemm_bench.py --set verdict &&
AKAP_PGEMM_GM=4 run l2_gm4 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/l2_gm4 -o run -- python3 tools/gemm_l2_probe.py &&
echo done
