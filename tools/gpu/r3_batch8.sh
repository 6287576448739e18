# round 3, batch 8: P/D chunked vs whole-prompt KV push on ONE GPU (2 ranks sharing it, gloo
# host-staged KV channel): 4096-token prompts prefilled in 1024-token chunks, so a streamed
# prompt's first 3 chunks of KV move while its last chunk is computed
set -o pipefail
mkdir -p gpurun_out/pd
for push in chunked whole; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
    bench.py --gpus 2 --mode pd --dist-backend gloo --pd-push $push --input-len 4096 --output-len 16 \
    --num-requests 16 --max-num-batched-tokens 1024 --max-model-len 4608 --steps 2 --warmup 1 \
    > gpurun_out/pd/$push.log 2>&1 || exit 1
done
