# round 6: the opening prefill phase of the headline bench, step by step (kernel trace)
set -u
O=gpurun_out/s9zb; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run prof 600 rocprofv3 --kernel-trace -d /tmp/pp -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 1 &&
run phase 120 python3 tools/prefill_phase.py /tmp/pp/run_kernel_trace.csv &&
echo done
