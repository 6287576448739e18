#!/usr/bin/env python3
"""Where the headline bench's TTFT goes: the steps of each wave's opening prefill phase, from a
rocprofv3 --kernel-trace CSV of `bench.py` (round 6).

A step ends at its sampling launch (argmax / sample kernel).  For every step from the first
prefill-attention launch of a wave until its first pure-decode stretch, the table lists the
step's GPU span (first dispatch start -> sampling end), the GPU time inside it (sum of kernel
durations), the idle gap before it (previous step's end -> this step's first dispatch: the
host's scheduling + launch time), its prefill-attention launches and whether decode rows rode
along (decode-attention launches).

    python tools/prefill_phase.py run_kernel_trace.csv [--waves 2]
"""
import argparse
import csv
import sys


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--waves", type=int, default=2)
    a = ap.parse_args()
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(a.trace)))
    steps, cur = [], []
    for r in rows:
        cur.append(r)
        if "argmax_kernel" in r[2] or "sample_kernel" in r[2]:
            steps.append(cur)
            cur = []
    waves, i = [], 0
    while i < len(steps) and len(waves) < a.waves + 8:
        if any("prefill_fa" in r[2] for r in steps[i]):
            j = i
            while j < len(steps) and (any("prefill_fa" in r[2] for r in steps[j])
                                      or j - i < 2):
                j += 1
            waves.append((i, j))
            # skip this wave's decode stretch
            while j < len(steps) and not any("prefill_fa" in r[2] for r in steps[j]):
                j += 1
            i = j
        else:
            i += 1
    for w, (i, j) in enumerate(waves[-a.waves:]):
        t0 = steps[i][0][0]
        print(f"## wave {w}: steps {i}..{j - 1}")
        print("| step | starts at ms | gap before us | span ms | GPU busy ms | prefill attn | "
              "decode attn | dispatches |")
        print("|---:|---:|---:|---:|---:|---:|---:|---:|")
        prev_end = steps[i - 1][-1][1] if i > 0 else steps[i][0][0]
        for k in range(i, j):
            s = steps[k]
            busy = sum(e - b for b, e, _ in s) / 1e6
            npf = sum("prefill_fa" in r[2] for r in s)
            ndc = sum("paged_attn_decode" in r[2] for r in s)
            print(f"| {k} | {(s[0][0] - t0) / 1e6:.2f} | {(s[0][0] - prev_end) / 1e3:.1f} | "
                  f"{(s[-1][1] - s[0][0]) / 1e6:.2f} | {busy:.2f} | {npf} | {ndc} | {len(s)} |")
            prev_end = s[-1][1]
        print()
        s = steps[i]
        big = sorted(((s[k + 1][0] - s[k][1], k) for k in range(len(s) - 1)), reverse=True)[:8]
        print(f"largest GPU-idle gaps inside step {i} (us, previous -> next kernel):")
        for g, k in sorted(big, key=lambda x: x[1]):
            print(f"  #{k:4d} {g / 1e3:9.1f}  {s[k][2][:60]} -> {s[k + 1][2][:60]}")
        print()
    return 0


if __name__ == "__main__":
    sys.exit(main())
