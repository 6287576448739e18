set -u
O=gpurun_out/r4p; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
run tk 300 $P tests/test_kernels_gpu.py -k "moe or router" &&
run te 300 $P tests/test_engine_gpu.py -k "moe or mixtral or hand_written" &&
run qwen3moe 600 python -u bench.py --model qwen3-30b-a3b --steps 2 &&
run mixtral 600 python -u bench.py --model mixtral-8x7b --num-requests 128 --max-num-seqs 128 --steps 1
echo done
