# pgemm vs hipBLASLt: kernel trace (resources) + PMC passes; Llama-3-8B P/D over IPC
set -u
O=gpurun_out/r4d; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ]; }
PM="python3 tools/pgemm_pmc_probe.py"
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
AKAP_PGEMM_V=33 run t33 200 $P tests/test_kernels_gpu.py -k pgemm &&
AKAP_PGEMM_V=34 run t34 200 $P tests/test_kernels_gpu.py -k pgemm &&
AKAP_PGEMM_V=43 run t43 200 $P tests/test_kernels_gpu.py -k pgemm &&
AKAP_PGEMM_V=44 run t44 200 $P tests/test_kernels_gpu.py -k pgemm &&
AKAP_PGEMM_V=33 run b33 300 python -u tools/pgemm_bench.py &&
AKAP_PGEMM_V=43 run b43 300 python -u tools/pgemm_bench.py &&
AKAP_PGEMM_V=44 run b44 300 python -u tools/pgemm_bench.py &&
AKAP_PGEMM_V=34 run b34 300 python -u tools/pgemm_bench.py &&
run b1 300 python -u tools/pgemm_bench.py &&
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
C2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE GRBM_COUNT"
run kt_pg 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_pg -o run -- $PM &&
run kt_lib 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_lib -o run -- $PM --lib &&
run p1_pg 90 rocprofv3 --pmc $C1 --output-format csv -d $O/p1_pg -o run -- $PM &&
run p1_lib 90 rocprofv3 --pmc $C1 --output-format csv -d $O/p1_lib -o run -- $PM --lib &&
run p2_pg 90 rocprofv3 --pmc $C2 --output-format csv -d $O/p2_pg -o run -- $PM &&
run p2_lib 90 rocprofv3 --pmc $C2 --output-format csv -d $O/p2_lib -o run -- $PM --lib &&
run pd_llama 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --mode pd --model llama-3-8b --dist-backend gloo --kv-transport ipc --gpus 1
echo done
