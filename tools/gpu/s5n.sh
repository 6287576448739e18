# sampler filter passes (fewer, larger chunks; pass A split out); EP=2 rehearsal with the new
# dispatch layout; then the whole kernel test file
set -u
O=gpurun_out/s5n; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run samp_t 300 $P tests/test_kernels_gpu.py -k "sampl or argmax" &&
run samp_b 300 python -u tools/sample_bench.py &&
AKAP_MOE_MODE=ep run ep2 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29623 bench.py --tp 2 --model qwen3-30b-a3b --dist-backend gloo --gpus 1 --steps 2 --warmup 1 &&
run tp_ep 500 $P tests/test_tp_gpu.py &&
run kernels 900 $P tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py &&
echo done
