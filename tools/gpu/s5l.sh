# sampler with batched sc1 loads in the filter passes (tests + microbench); EP=2 Qwen3-MoE
# rehearsal kernel table (bench --torch-profile on rank 0); clean T=1.0 kernel table of the
# headline bench (GEMM plan from a tuning cache: no tuner launches in the profiled run)
set -u
O=gpurun_out/s5l; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run pd1p2d 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --mode pd --pd-prefill-ranks 1 --dist-backend gloo --steps 2 &&
run samp_t 300 $P tests/test_kernels_gpu.py -k "sampl or argmax" &&
run samp_b 300 python -u tools/sample_bench.py &&
AKAP_MOE_MODE=ep run ep2_prof 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29623 bench.py --tp 2 --model qwen3-30b-a3b --dist-backend gloo --gpus 1 --steps 1 --warmup 1 --output-len 8 --torch-profile &&
export AKAP_GEMM_TUNE_CACHE=/tmp/tune_qwen3.json &&
run tunecache 400 python -u bench.py --steps 1 --warmup 0 &&
run prof_t1 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt1 -o run -- python3 bench.py --temperature 1.0 --steps 1 --warmup 1 &&
python3 tools/prof_summary.py /tmp/pt1/run_kernel_stats.csv > $O/t1_kernel_stats.md && rm -rf /tmp/pt1 &&
echo done
