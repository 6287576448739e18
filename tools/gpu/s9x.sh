# round 6: serving prefill attention with / without the longest-first tile map (kernel traces)
set -u
O=gpurun_out/s9x; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run apq 300 python -u tools/attn_prefill_probe.py --only qwen3-0.6b:32x512 --qprep &&
PROBE_UNSORTED=1 run apq_unsorted 300 python -u tools/attn_prefill_probe.py --only qwen3-0.6b:32x512 --qprep &&
run prof1 600 rocprofv3 --kernel-trace --stats -d /tmp/p1 -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 1 &&
run prof1_s 120 python3 tools/prof_summary.py /tmp/p1/run_kernel_trace.csv $O/prof1.md "sorted tile map" &&
AKAP_TILE_SORT=0 run prof0 600 rocprofv3 --kernel-trace --stats -d /tmp/p0 -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 1 &&
run prof0_s 120 python3 tools/prof_summary.py /tmp/p0/run_kernel_trace.csv $O/prof0.md "map order" &&
cp /tmp/p1/run_kernel_trace.csv /tmp/p1.csv && python3 - <<'PY' > $O/prefill_steps.log
import csv
for tag in ("p1", "p0"):
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(f"/tmp/{tag}/run_kernel_trace.csv")))
    att = [(e - s) / 1e3 for s, e, n in rows if "prefill_fa" in n]
    print(tag, "prefill attn calls", len(att), "mean us %.1f" % (sum(att) / max(1, len(att))),
          "first 28: %.1f" % (sum(att[:28]) / 28 if len(att) >= 28 else 0))
PY
echo done
