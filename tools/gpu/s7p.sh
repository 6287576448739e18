# idle gaps in the headline bench's kernel trace (prefill vs decode windows)
set -u
O=gpurun_out/s7p; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run trace 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt -o run -- python3 bench.py --steps 1 --warmup 1 &&
python3 tools/trace_gaps.py /tmp/kt --min-us 5 --top 25 > $O/gaps.txt 2>&1 &&
echo done
