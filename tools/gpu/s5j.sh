# hipIpc multi-importer probes, continued (s5g: 12 x 6.6 GiB segments hang when the importers
# already hold 79 GiB each).  Does opening BEFORE the importers' own allocation work?  Does a
# smaller own allocation work?  First hang ends the call.
set -u
O=gpurun_out/s5j; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
Q="python -u tools/ipc_multi_open_probe.py --world 3 --mode serial"
run s3_f79_first 90 $Q --gb 79 --segments 3 --fill 79 --open-first &&
run s3_f20 90 $Q --gb 79 --segments 3 --fill 20 &&
run s3_f40 90 $Q --gb 40 --segments 3 --fill 40 &&
echo done
