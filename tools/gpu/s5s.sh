# sampler filter passes with wave-aggregated histogram adds; model refreshes on the final tree:
# Llama-3-8B monolithic, Llama-3-8B P/D (prefill + decode processes, hipIpc pull), Mixtral-8x7B
set -u
O=gpurun_out/s5s; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run samp_t 300 $P tests/test_kernels_gpu.py -k "sampl or argmax" &&
run samp_b 300 python -u tools/sample_bench.py &&
run t64 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/st64 -o run -- python3 tools/sample_pass_probe.py --B 64 &&
python3 tools/sample_pass_probe.py --summarize /tmp/st64/run_kernel_trace.csv > $O/b64.txt &&
run llama8b 600 python -u bench.py --model llama-3-8b --steps 2 &&
run pd_llama8b 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --mode pd --model llama-3-8b --dist-backend gloo --kv-transport ipc --gpus 1 --steps 2 &&
run mixtral 900 python -u bench.py --model mixtral-8x7b --num-requests 128 --steps 2 &&
echo done
