# round 5 baseline: headline bench writing a GEMM tune cache, then a clean rocprofv3 kernel
# trace of the serving step from that cache (no tuner launches), then the GEMM microbenches
set -u
O=gpurun_out/s5a; mkdir -p $O
export AKAP_GEMM_TUNE_CACHE=$PWD/$O/tune_qwen3.json
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run bench 600 python -u bench.py &&
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null &&
run prof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u bench.py --steps 1 --warmup 1 &&
run m256 400 python -u tools/gemm_m256.py &&
run pgemm 400 python -u tools/pgemm_bench.py --json $O/pgemm.json &&
echo done
