# round 6: hipIpc hang bisection 1: HIP importers with unwritten memory; then ONE torch importer
# (world 2) at the round-5 sizes (LAST: may hang until its SIGALRM deadline)
set -u
O=gpurun_out/s9e; mkdir -p $O
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
SWEEP_OUT=$O FILL=0 POINTS="2:79:79:6.6:0 1:79:79:6.6:0" run hip_nofill 300 bash tools/gpu/s9_ipc_sweep2.sh &&
run torch_w2 150 python -u tools/ipc_multi_open_probe.py --mode concurrent --gb 79 --world 2 --fill 79 --segments 12 --deadline 100 &&
echo done
