# round 6: step-start idle distribution of the headline decode steps (kernel trace)
set -u
O=gpurun_out/s9zk; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run prof 600 rocprofv3 --kernel-trace -d /tmp/pk -o run --output-format csv -- python3 -u bench.py --steps 2 --warmup 1 &&
run bounds 120 python3 tools/decode_boundaries.py /tmp/pk/run_kernel_trace.csv &&
echo done
