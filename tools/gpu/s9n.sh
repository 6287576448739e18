# round 6: stream-first pgemm as the default: GEMM + engine GPU tests, then same-box headline
# A/B against the phase pipeline (AKAP_PGEMM_SCHED=1), Llama-3-8B and Mixtral with the default
set -u
O=gpurun_out/s9n; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run t_gemm 400 $P tests/test_kernels_gpu.py tests/test_fused_decode.py -k "pgemm or gemm or moe" &&
run t_engine 400 $P tests/test_engine_gpu.py &&
run b4a 400 python -u bench.py &&
AKAP_PGEMM_SCHED=1 run b1a 400 python -u bench.py &&
run b4b 400 python -u bench.py &&
AKAP_PGEMM_SCHED=1 run b1b 400 python -u bench.py &&
run l8 900 python -u bench.py --model llama-3-8b &&
AKAP_PGEMM_SCHED=1 run l8s1 900 python -u bench.py --model llama-3-8b &&
echo done
