set -u
O=gpurun_out/r4l; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
run t4 200 $P tests/test_kernels_gpu.py -k pgemm &&
AKAP_PGEMM_NB=2 run t2 200 $P tests/test_kernels_gpu.py -k pgemm &&
run b4 300 python -u tools/pgemm_bench.py &&
AKAP_PGEMM_NB=2 run b2 300 python -u tools/pgemm_bench.py &&
ROCP_TOOL_LIBRARIES=$PWD/aws_k8s_ansible_provisioner_amd/libakap_pmc.so run pmc 120 python -u tools/pmc_probe.py &&
run metrics 300 python -u tools/metrics_load_probe.py --out gpurun_out/r4l/metrics &&
AKAP_BENCH_STACKS=100 run pd12 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29613 bench.py --mode pd --pd-prefill-ranks 1 --dist-backend gloo --kv-transport p2p --gpus 1
echo done
