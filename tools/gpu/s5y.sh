# IPC all-to-all / all-gather unroll: correctness tests + A/B timing vs the previous .so
set -u
O=gpurun_out/s5y; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
mkdir -p /tmp/old && cp -r aws_k8s_ansible_provisioner_amd /tmp/old/ && cp tools/gpu/_C_old.so /tmp/old/aws_k8s_ansible_provisioner_amd/_C.so &&
true &&
AKAP_REPO_ROOT=/tmp/old AKAP_ALLOW_STALE_NATIVE=1 run old2 200 python -u tools/car_bench.py --world 2 &&
run new2 200 python -u tools/car_bench.py --world 2 &&
AKAP_REPO_ROOT=/tmp/old AKAP_ALLOW_STALE_NATIVE=1 run old4 200 python -u tools/car_bench.py --world 4 &&
run new4 200 python -u tools/car_bench.py --world 4 &&
echo done
