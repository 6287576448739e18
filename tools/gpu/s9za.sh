# round 6: prefill tile rows A/B on one box (engine default vs forced), Qwen3 and Llama-3-8B
set -u
O=gpurun_out/s9za; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run q_def_a 400 python -u bench.py &&
AKAP_PREFILL_TILE_ROWS=256 run q_256_a 400 python -u bench.py &&
run q_def_b 400 python -u bench.py &&
AKAP_PREFILL_TILE_ROWS=256 run q_256_b 400 python -u bench.py &&
run l_def_a 600 python -u bench.py --model llama-3-8b &&
AKAP_PREFILL_TILE_ROWS=128 run l_128_a 600 python -u bench.py --model llama-3-8b &&
echo done
