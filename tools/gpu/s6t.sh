# qk_norm_rope_cache: token-major q/k role vs the (token, head) form (previous .so)
set -u
O=gpurun_out/s6t; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
mkdir -p /tmp/old && cp -r aws_k8s_ansible_provisioner_amd /tmp/old/ && cp tools/gpu/_C_prev.so /tmp/old/aws_k8s_ansible_provisioner_amd/_C.so &&
run t_rope 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "rope or prefill or attn" &&
run new 200 python -u tools/rope_probe.py &&
mkdir -p /tmp/old/tools && cp tools/rope_probe.py /tmp/old/tools/ &&
AKAP_ALLOW_STALE_NATIVE=1 run old 200 python -u /tmp/old/tools/rope_probe.py &&
echo done
