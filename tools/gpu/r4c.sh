set -u
O=gpurun_out/r4c; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
P="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
TR="python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611"
run pgemm 300 $P tests/test_kernels_gpu.py -k pgemm &&
run pgbench 300 python -u tools/pgemm_bench.py --json $O/pgemm.json &&
ROCP_TOOL_LIBRARIES=$PWD/aws_k8s_ansible_provisioner_amd/libakap_pmc.so run pmc 120 python -u tools/pmc_probe.py &&
run pd_qwen 420 $TR bench.py --mode pd --dist-backend gloo --kv-transport ipc --gpus 1 &&
run pd_llama 900 $TR bench.py --mode pd --model llama-3-8b --dist-backend gloo --kv-transport ipc --gpus 1 &&
run rehearsal70b 600 python -u bench/tp_shard_rehearsal.py --B 64,256
echo done
