# round 6: decode-GEMM ingress probe with a per-workgroup K stagger (StaggerU-style)
set -u
O=gpurun_out/s8c; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run ingress 300 ./tools/probes/ingress_probe "" 30 &&
echo done
