# (A/B harness: abso/_C_old.so = HEAD, abso/_C_new.so = decode kernel at __launch_bounds__(256, 2);
#  both built locally and removed afterwards)
set -u
O=gpurun_out/s9zq; mkdir -p $O
P=aws_k8s_ansible_provisioner_amd
for v in old new old new; do
  cp abso/_C_$v.so $P/_C.so
  AKAP_ALLOW_STALE_NATIVE=1 timeout -k 10 200 python -u bench/attn_fused_ab.py > $O/ab_$v.log 2>&1 || exit 1
  echo "$v: $(grep -E 'serving|q ready' $O/ab_$v.log | tr '\n' ' ')"
done
cp abso/_C_new.so $P/_C.so
AKAP_ALLOW_STALE_NATIVE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_decode.py -k "decode" > $O/t.log 2>&1; echo "tests rc=$? $(tail -1 $O/t.log)"
for v in old new; do
  cp abso/_C_$v.so $P/_C.so
  AKAP_ALLOW_STALE_NATIVE=1 timeout -k 10 400 python -u bench.py > $O/b_$v.log 2>&1 || exit 1
  echo "bench $v: $(grep -o '"value": [0-9.]*\|"p50_ttft_ms": [0-9.]*' $O/b_$v.log | tr '\n' ' ')"
done
cp abso/_C_new.so $P/_C.so
