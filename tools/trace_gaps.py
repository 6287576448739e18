#!/usr/bin/env python3
"""GPU idle gaps from a rocprofv3 --kernel-trace CSV (*_kernel_trace.csv): per step kind
(prefill steps = the span from a step's first prefill-attention launch's layer back to its
sampling; decode = the rest), total busy time, total gap time, and the largest gaps with the
kernels on either side.

    python tools/trace_gaps.py DIR_OR_CSV [--min-us 5] [--top 15]
"""
import csv
import glob
import os
import sys


def main():
    src = sys.argv[1]
    min_us = float(sys.argv[sys.argv.index("--min-us") + 1]) if "--min-us" in sys.argv else 5.0
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 15
    path = src if src.endswith(".csv") else glob.glob(os.path.join(src, "**", "*kernel_trace.csv"),
                                                      recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # a prefill window opens at the first qk_norm_rope / prefill attention launch after a
    # sampling launch and closes at the next sampling launch
    gaps = {"prefill": [], "decode": []}
    busy = {"prefill": 0, "decode": 0}
    mode = "decode"
    end = rows[0][1]
    for i, (s, e, n) in enumerate(rows):
        if "prefill_fa" in n:
            mode = "prefill"
        g = s - end
        if i and g > min_us * 1e3:
            gaps[mode].append((g, rows[i - 1][2][:60], n[:60]))
        busy[mode] += e - s
        end = max(end, e)
        if "argmax_kernel" in n or "sample_" in n:
            mode = "decode"
    for k in ("prefill", "decode"):
        tot = sum(g for g, _, _ in gaps[k])
        print(f"{k}: busy {busy[k] / 1e6:.1f} ms, gaps > {min_us} us: {len(gaps[k])} totalling "
              f"{tot / 1e6:.2f} ms")
        for g, a, b in sorted(gaps[k], reverse=True)[:top]:
            print(f"   {g / 1e3:9.1f} us  after {a}  before {b}")


if __name__ == "__main__":
    main()
