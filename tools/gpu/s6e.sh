# sampler chunk-count sweep (AKAP_SAMPLE_CHUNKS diagnostic override)
set -u
O=gpurun_out/s6e; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
for S in 2 4 8 16 38 64; do AKAP_SAMPLE_CHUNKS=$S run s$S 200 python -u tools/sample_bench.py || exit 1; done
echo done
