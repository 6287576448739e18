# decode attention after the prologue-preload + named double-buffer rework: numerics, micro,
# fused-vs-plain micro, headline bench (default and the 3-WG/CU variant), kernel stats
set -o pipefail
mkdir -p gpurun_out/ab3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "decode or v_tail" > gpurun_out/ab3/tests.log 2>&1 && \
timeout -k 10 120 python -u bench/attn_micro.py --B 256 --ctx 640 --spread 0 --parts 1 > gpurun_out/ab3/attn_micro.log 2>&1 && \
timeout -k 10 120 python -u bench/attn_micro.py --B 32 --ctx 2048 --spread 0 --parts 1 >> gpurun_out/ab3/attn_micro.log 2>&1 && \
timeout -k 10 120 python -u bench/attn_fused_ab.py > gpurun_out/ab3/fused_ab.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab3/bench_65.log 2>&1 && \
AKAP_ATTN_FLAGS=321 AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab3/bench_321.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab3/bench_65b.log 2>&1 && \
AKAP_KGEMM_NS=5 AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 300 python -u bench.py --steps 2 > gpurun_out/ab3/bench_kns5.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab3/prof -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/ab3/bench_prof.log 2>&1
