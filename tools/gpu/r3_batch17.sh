# round 3, batch 17: online serving (Poisson arrivals -> mixed prefill+decode steps, V tail on the
# writer + plain-decode path) and a saturated online run; fp8-KV headline for reference
set -o pipefail
mkdir -p gpurun_out/on
timeout -k 10 400 python -u bench.py --arrival-rate 100 --steps 1 --warmup 1 > gpurun_out/on/poisson100.log 2>&1 && \
timeout -k 10 400 python -u bench.py --arrival-rate 100 --max-num-seqs 64 --steps 1 --warmup 1 > gpurun_out/on/sat64.log 2>&1 && \
timeout -k 10 300 python -u bench.py --kv-cache-dtype fp8 --steps 2 > gpurun_out/on/fp8kv.log 2>&1
