set -u
O=gpurun_out/r4a; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
P="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
run car 420 $P tests/test_custom_allreduce_gpu.py -k "ipc or pull or siblings" &&
run attn 600 $P tests/test_kernels_gpu.py -k "attention or v_tail or kv" &&
run pdtp 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_pd_gpu.py tests/test_tp_gpu.py &&
run bench 600 python -u bench.py &&
run pgemm 300 $P tests/test_kernels_gpu.py -k pgemm &&
run pgeng 300 $P tests/test_engine_gpu.py -k hand_written &&
run pgbench 300 python -u tools/pgemm_bench.py --json $O/pgemm.json &&
AKAP_PREFILL_GEMM=pgemm run bench_pg 600 python -u bench.py &&
ROCP_TOOL_LIBRARIES=$PWD/aws_k8s_ansible_provisioner_amd/libakap_pmc.so run pmc 120 python -u tools/pmc_probe.py
echo done
