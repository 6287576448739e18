# round 6: hipIpc hang bisection 3 (torch-bundled ROCm 7.0.2 runtime): which size triggers it --
# the export alone (X = 0), the importer's own allocation alone, or their sum?  Stops at the
# first hang.
set -u
O=gpurun_out/s9g; mkdir -p $O
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
TL=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
SWEEP_OUT=$O/torchrt IPC_REPRO_HIPLIB=$TL/libamdhip64.so POINTS="${POINTS:-1:0:40:6.6:0 1:40:8:6.6:0 1:0:72:6.6:0 1:72:8:6.6:0 1:36:36:6.6:0}" run torchrt 600 bash tools/gpu/s9_ipc_sweep2.sh &&
echo done
