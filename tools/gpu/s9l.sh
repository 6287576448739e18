# round 6: stream-first pgemm body (AKAP_PGEMM_SCHED=4): correctness, then the verdict shape set
set -u
O=gpurun_out/s9l; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
AKAP_PGEMM_SCHED=4 run t_pg4 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k pgemm &&
AKAP_PGEMM_SCHED=4 run pg4 300 python -u tools/pgemm_bench.py --set verdict &&
run pg1 300 python -u tools/pgemm_bench.py --set verdict &&
echo done
