# Online serving (Poisson arrivals) with mixed vs prefill-first scheduling + the burst headline.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
set -e
B="timeout -k 10 240 python3 bench.py --steps 1 --warmup 1 --num-requests 400 --arrival-rate 100"
$B --max-num-batched-tokens 4096 > gpurun_out/r2_online_mixed_4k.log 2>&1
$B --max-num-batched-tokens 4096 --no-mixed-batching > gpurun_out/r2_online_pfirst_4k.log 2>&1
$B > gpurun_out/r2_online_mixed_16k.log 2>&1
$B --no-mixed-batching > gpurun_out/r2_online_pfirst_16k.log 2>&1
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > gpurun_out/r2_bench_b.log 2>&1
echo online ok
