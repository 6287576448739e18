# round 6: down-projection split-K forms, timing + counters (one PMC pass per block set)
set -u
O=gpurun_out/s9c; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run warmth 300 python -u tools/weight_warmth_probe.py &&
run pmc1 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS -d $O/pmc1 -o run --output-format csv -- python3 -u tools/weight_warmth_probe.py &&
run pmc2 120 rocprofv3 --kernel-trace --stats --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d $O/pmc2 -o run --output-format csv -- python3 -u tools/weight_warmth_probe.py &&
echo done
