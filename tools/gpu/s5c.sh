# sampler v2 (sc1 publish, filter kernel) tests + bench; pgemm 4-wave 128x128 form vs 8-wave
set -u
O=gpurun_out/s5c; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run samp_t 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sampl or argmax" &&
run samp_b 300 python -u tools/sample_bench.py &&
AKAP_PGEMM_WAVES=4 run pg4_t 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pgemm" &&
run pg8_b 400 python -u tools/pgemm_bench.py --json $O/pg8.json &&
AKAP_PGEMM_WAVES=4 run pg4_b 400 python -u tools/pgemm_bench.py --json $O/pg4.json &&
AKAP_PGEMM_WAVES=4 run sk4_b 400 python -u tools/pgemm_m256_probe.py &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
echo done
