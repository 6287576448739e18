# sampler with unrolled row visits: tests, microbench, per-launch pass durations at B = 64
set -u
O=gpurun_out/s5p; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run samp_t 300 $P tests/test_kernels_gpu.py -k "sampl or argmax" &&
run samp_b 300 python -u tools/sample_bench.py &&
run t64 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/st64 -o run -- python3 tools/sample_pass_probe.py --B 64 &&
python3 tools/sample_pass_probe.py --summarize /tmp/st64/run_kernel_trace.csv > $O/b64.txt &&
echo done
