# round 6: stream-first pgemm, 4-wave form and raster height, same box
set -u
O=gpurun_out/s9m; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
AKAP_PGEMM_SCHED=4 AKAP_PGEMM_WAVES=4 run t_pg4w4 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k pgemm &&
AKAP_PGEMM_SCHED=4 AKAP_PGEMM_WAVES=4 run pg4w4 300 python -u tools/pgemm_bench.py --set verdict &&
AKAP_PGEMM_SCHED=4 run pg4w8 300 python -u tools/pgemm_bench.py --set verdict &&
AKAP_PGEMM_SCHED=4 AKAP_PGEMM_GM=4 run pg4w8gm4 300 python -u tools/pgemm_bench.py --set verdict &&
echo done
