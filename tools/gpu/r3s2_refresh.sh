# refresh the other model families on the final kernels: 70B TP=8 rank-shard rehearsal, Mixtral 1-GPU bench
set -o pipefail
mkdir -p gpurun_out/rf
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u bench/tp_shard_rehearsal.py --model llama-3-70b --tp 8 --B 64,128,256 --ctx 1024 > gpurun_out/rf/llama70b_tp8_rank.log 2>&1 && \
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --num-requests 128 --max-num-seqs 128 --steps 1 > gpurun_out/rf/mixtral.log 2>&1
