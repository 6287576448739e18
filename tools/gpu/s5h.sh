# sampler v3 (inverse-CDF T>0 draw, distributed top-k/top-p passes): tests + microbench;
# TP=4 at Llama-3-70B widths, decode per-step time at B=256 with prefill chunks that keep every
# all-reduce on the one-shot/two-shot IPC kernel (<= 8 MiB, no piecewise path)
set -u
O=gpurun_out/s5h; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run samp_t 300 $P tests/test_kernels_gpu.py -k "sampl or argmax" &&
run samp_b 300 python -u tools/sample_bench.py &&
run samp_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sp -o run -- python3 tools/sample_bench.py &&
python3 tools/prof_summary.py /tmp/sp/run_kernel_stats.csv > $O/samp_kernel_stats.md && rm -rf /tmp/sp &&
run tp4_70b_bench 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29624 bench.py --tp 4 --model llama-3-70b-l4 --dist-backend gloo --gpus 1 --steps 1 --warmup 1 --input-len 1024 --output-len 64 --max-num-batched-tokens 512 &&
echo done
