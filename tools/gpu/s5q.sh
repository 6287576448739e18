# PMC of the sampler's filter passes at B = 64 (top-k 50 + top-p 0.9): where does pass A's time
# go (LDS atomics, waits, VALU)?  Counter passes in separate runs (no traces combined)
set -u
O=gpurun_out/s5q; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
C1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
C2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS GRBM_COUNT"
run p1 90 rocprofv3 --pmc $C1 --output-format csv -d /tmp/q1 -o run -- python3 tools/sample_pass_probe.py --B 64 --iters 10 &&
run p2 90 rocprofv3 --pmc $C2 --output-format csv -d /tmp/q2 -o run -- python3 tools/sample_pass_probe.py --B 64 --iters 10 &&
python3 tools/pmc_summary.py $O/samp_pmc.md "sampler passes B=64" /tmp/q1/run_counter_collection.csv /tmp/q2/run_counter_collection.csv --match sample > $O/summ.log 2>&1 &&
cp /tmp/q1/run_counter_collection.csv $O/q1.csv && cp /tmp/q2/run_counter_collection.csv $O/q2.csv &&
echo done
