# sampler: distributed B/C restored, per-slot window atomics; + flat top-p (fallback) case
set -u
O=gpurun_out/s6s; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run t_samp 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "sampl or argmax" &&
run bench 300 python -u tools/sample_bench.py &&
run t64 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/st64 -o run -- python3 tools/sample_pass_probe.py --B 64 &&
python3 tools/sample_pass_probe.py --summarize /tmp/st64/run_kernel_trace.csv > $O/b64.txt &&
run t256 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/st256 -o run -- python3 tools/sample_pass_probe.py --B 256 &&
python3 tools/sample_pass_probe.py --summarize /tmp/st256/run_kernel_trace.csv > $O/b256.txt &&
echo done
