# prefill attention with the fused q prep (AKAP_PREFILL_QPREP): kernel tests, engine tests,
# smoke, headline bench A/B, kernel table of one bench
set -u
O=gpurun_out/s7l; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run t_attn 300 $P tests/test_kernels_gpu.py -k "prefill or attn or qk_norm or rope" &&
run t_engine 400 $P tests/test_engine_gpu.py &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
run bench1 400 python -u bench.py --steps 3 --warmup 1 &&
AKAP_PREFILL_QPREP=0 run bench0 400 python -u bench.py --steps 3 --warmup 1 &&
run bench1b 400 python -u bench.py --steps 3 --warmup 1 &&
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf -o run -- python3 bench.py --steps 1 --warmup 1 &&
python3 tools/prof_summary.py /tmp/pf/run_kernel_stats.csv > $O/kernel_stats.md &&
echo done
