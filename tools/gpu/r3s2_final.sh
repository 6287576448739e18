# round-3 session-2 verification: full GPU suite, smoke, headline bench (+ kernel stats and step
# gaps of the steady state), Llama-3-8B bench
set -o pipefail
mkdir -p gpurun_out/fin
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fin/gputests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 400 python -u bench.py > gpurun_out/fin/bench.log 2>&1 && \
AKAP_GEMM_TUNE_CACHE=/tmp/tune.json timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin/prof -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/fin/bench_prof.log 2>&1 && \
timeout -k 10 500 python -u bench.py --model llama-3-8b --steps 2 > gpurun_out/fin/llama8b.log 2>&1
