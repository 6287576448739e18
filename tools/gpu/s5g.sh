# hipIpc multi-importer probe matrix, 3 processes on one GPU (the 1P:2D P/D layout): does the
# open hang depend on the segment size, on the importers' own allocations, or on both?  Smallest
# first; the first hang ends the call (each probe bounded)
set -u
O=gpurun_out/s5g; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
Q="python -u tools/ipc_multi_open_probe.py --world 3 --mode serial"
run s12_f79 90 $Q --gb 79 --segments 12 --fill 79 &&
run s3_f40 90 $Q --gb 40 --segments 3 --fill 40 &&
run s6_f79 90 $Q --gb 79 --segments 6 --fill 79 &&
run s3_f79 90 $Q --gb 79 --segments 3 --fill 79 &&
echo done
