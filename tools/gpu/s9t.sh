# round 6: pgemm SCHED 5 (split-step stream-first: fragment reads under the other step's MFMAs)
set -u
O=gpurun_out/s9t; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
AKAP_PGEMM_SCHED=5 run t_pg5 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k pgemm &&
AKAP_PGEMM_SCHED=5 run pg5 300 python -u tools/pgemm_bench.py --set verdict &&
run pg4 300 python -u tools/pgemm_bench.py --set verdict &&
echo done
