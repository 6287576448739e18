# KV block size A/B (32 default vs 64) on the headline bench; micro at BS 64
set -o pipefail
mkdir -p gpurun_out/bs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python -u bench/attn_micro.py --B 256 --ctx 640 --spread 0 --parts 1 --bs 32 > gpurun_out/bs/micro.log 2>&1 && \
timeout -k 10 120 python -u bench/attn_micro.py --B 256 --ctx 640 --spread 0 --parts 1 --bs 64 >> gpurun_out/bs/micro.log 2>&1 && \
timeout -k 10 120 python -u bench/attn_micro.py --B 256 --ctx 640 --spread 0 --parts 1 --bs 128 >> gpurun_out/bs/micro.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tq.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/bs/q32.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tq.json timeout -k 10 300 python -u bench.py --steps 2 --block-size 64 > gpurun_out/bs/q64.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tq.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/bs/q32b.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tq.json timeout -k 10 300 python -u bench.py --steps 2 --block-size 64 > gpurun_out/bs/q64b.log 2>&1
