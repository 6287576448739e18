# round 6: hipIpc hang bisection 2: the HIP-runtime-only reproducer on the runtime PyTorch
# bundles (ROCm 7.0.2, what every engine process uses) vs /opt/rocm (7.2), one importer,
# growing sizes; the sweep stops at the first hang
set -u
O=gpurun_out/s9f; mkdir -p $O
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
TL=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
SWEEP_OUT=$O/rocm72 POINTS="1:79:79:6.6:0" run rocm72 200 bash tools/gpu/s9_ipc_sweep2.sh &&
SWEEP_OUT=$O/torchrt IPC_REPRO_HIPLIB=$TL/libamdhip64.so POINTS="1:8:8:4:0 1:32:32:32:0 1:48:48:6.6:0 1:64:64:6.6:0 1:79:79:6.6:0" run torchrt 600 bash tools/gpu/s9_ipc_sweep2.sh &&
echo done
