# sampler v2 (sc1 publish, filter kernel) tests + bench; kv_pull on plane tables (segmented
# caches); pgemm 4-wave 128x128 form vs 8-wave; smoke; 1P:2D P/D on one GPU over ipc
set -u
O=gpurun_out/s5c; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run samp_t 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sampl or argmax" &&
run samp_b 300 python -u tools/sample_bench.py &&
run kvpull 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_custom_allreduce_gpu.py -k "kv_pull" &&
AKAP_PGEMM_WAVES=4 run pg4_t 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pgemm" &&
run pg8_b 400 python -u tools/pgemm_bench.py --json $O/pg8.json &&
AKAP_PGEMM_WAVES=4 run pg4_b 400 python -u tools/pgemm_bench.py --json $O/pg4.json &&
AKAP_PGEMM_WAVES=4 run sk4_b 400 python -u tools/pgemm_m256_probe.py &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
run pd1p2d 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --mode pd --pd-prefill-ranks 1 --dist-backend gloo --steps 2 &&
echo done
