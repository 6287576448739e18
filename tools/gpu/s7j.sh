# PMC of the prefill attention kernel (8-wave 256-row tile and 4-wave 128-row tile) at the
# headline chunk (qwen3 32 x 512) and a long prompt (4 x 4096): where do the cycles go?
set -u
O=gpurun_out/s7j; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
C1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
C2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_COUNT"
for sh in qwen3-0.6b:32x512 qwen3-0.6b:4x4096; do
  for rows in 256 128; do
    t=${sh#*:}_$rows
    run a_$t 90 rocprofv3 --pmc $C1 --output-format csv -d /tmp/a_$t -o run -- python3 tools/attn_prefill_probe.py --only $sh --rows $rows || exit 1
    run b_$t 90 rocprofv3 --pmc $C2 --output-format csv -d /tmp/b_$t -o run -- python3 tools/attn_prefill_probe.py --only $sh --rows $rows || exit 1
    python3 tools/pmc_summary.py $O/pmc_$t.md "prefill attention $sh tile $rows" /tmp/a_$t/run_counter_collection.csv /tmp/b_$t/run_counter_collection.csv --match prefill_fa > $O/summ_$t.log 2>&1 || exit 1
  done
done
echo done
