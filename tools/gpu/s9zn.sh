# (A/B harness: abso/_C_old.so and abso/_C_new.so were built locally from HEAD~ and HEAD and removed afterwards)
set -u
O=gpurun_out/s9zn; mkdir -p $O
P=aws_k8s_ansible_provisioner_amd
for v in old new old new; do
  cp abso/_C_$v.so $P/_C.so
  AKAP_ALLOW_STALE_NATIVE=1 timeout -k 10 200 python -u tools/attn_prefill_probe.py --qprep --only qwen3-0.6b:32x512 > $O/ap_$v.log 2>&1 || exit 1
  echo "$v: $(grep qwen3 $O/ap_$v.log)"
done
cp abso/_C_new.so $P/_C.so
AKAP_ALLOW_STALE_NATIVE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill" > $O/t.log 2>&1; echo "tests rc=$? $(tail -1 $O/t.log)"
