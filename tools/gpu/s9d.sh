# round 6: hipIpc hang, HIP-only vs torch processes at the round-5 failing layout (1P:2D,
# 79 GiB export in 12 segments, each importer holding 79 GiB).  The torch probe runs LAST.
set -u
O=gpurun_out/s9d; mkdir -p $O
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
SWEEP_OUT=$O POINTS="2:79:79:6.6:0 2:88:88:6.6:0" run hip_single 300 bash tools/gpu/s9_ipc_sweep2.sh &&
run torch_small 150 python -u tools/ipc_multi_open_probe.py --mode concurrent --gb 8 --world 3 --fill 8 --segments 2 --deadline 100 &&
run torch_r5 150 python -u tools/ipc_multi_open_probe.py --mode concurrent --gb 79 --world 3 --fill 79 --segments 12 --deadline 100 &&
echo done
