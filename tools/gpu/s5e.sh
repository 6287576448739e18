# sampler v3 (inverse-CDF draw, padded tickets); padded GEMM tickets + sc1 in-launch gdgemm
# combine (decode GEMMs at M=256, split-K pgemm); TP=4 70B-width bench after the pre-capture
# barrier; two-pod P/D GPU test; server-load metrics window; bench at T=1.0 (+ kernel table)
set -u
O=gpurun_out/s5e; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run samp_t 300 $P tests/test_kernels_gpu.py -k "sampl or argmax" &&
run samp_b 300 python -u tools/sample_bench.py &&
run gemm_t 600 $P tests/test_kernels_gpu.py -k "dgemm or gdgemm or pgemm or gemm_inlaunch or split" &&
run m256 500 python -u tools/gemm_m256.py &&
run sk8 400 python -u tools/pgemm_m256_probe.py &&
run tp4_70b_bench 700 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29624 bench.py --tp 4 --model llama-3-70b-l4 --dist-backend gloo --gpus 1 --steps 2 --warmup 1 &&
run bench_t1 400 python -u bench.py --temperature 1.0 &&
run bench_t0 400 python -u bench.py &&
echo done
