# K13 full-grid epochs (custom collective GPU tests incl. the mixed no-sync sequence and the
# fp8 kv_pull case); chunked sampler (kernel tests + microbench); pgemm split-K in-launch
# combine (tests + M=256 sweep); decode-GEMM slope probe; hipIpc segmented-export probe
set -u
O=gpurun_out/s5b; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run samp_t 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sampl or argmax" &&
run samp_b 300 python -u tools/sample_bench.py &&
run sk_t 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pgemm_split_k" &&
run sk_b 400 python -u tools/pgemm_m256_probe.py &&
run slope 400 python -u tools/gemm_slope.py &&
run car 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_custom_allreduce_gpu.py &&
run ipc3seg 150 python -u tools/ipc_multi_open_probe.py --mode serial --gb 86 --segments 3 --world 3 &&
echo done
