# round 3, batch 18: saturated online run A/B (V tail on/off) and a repeat for variance
set -o pipefail
mkdir -p gpurun_out/on
timeout -k 10 400 python -u bench.py --arrival-rate 100 --max-num-seqs 64 --steps 1 --warmup 1 > gpurun_out/on/sat64_b.log 2>&1 && \
AKAP_V_TAIL=0 timeout -k 10 400 python -u bench.py --arrival-rate 100 --max-num-seqs 64 --steps 1 --warmup 1 > gpurun_out/on/sat64_notail.log 2>&1 && \
AKAP_ASYNC_DECODE=0 timeout -k 10 400 python -u bench.py --arrival-rate 100 --max-num-seqs 64 --steps 1 --warmup 1 > gpurun_out/on/sat64_sync.log 2>&1
