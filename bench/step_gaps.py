"""Idle GPU time inside and between decode steps from a rocprofv3 kernel trace.

For each window between two consecutive sampler launches (one decode step), sum the idle
gaps between consecutive kernels and report the largest one with the kernels around it:
the host's share of the step (D2H wait, scheduler, input staging, graph launch) shows up as
one long gap, launch latency inside the graph as many short ones.

python bench/step_gaps.py <run_kernel_trace.csv>
"""
import collections
import csv
import statistics
import sys


def short(n):
    n = n.replace("void akap::", "").replace("akap::", "")
    return n[:48]


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    samp = [i for i, r in enumerate(rows) if "sample_kernel" in r[2]]
    idle, big, busy, span = [], collections.Counter(), [], []
    for a, b in zip(samp, samp[1:]):
        tot, best = 0.0, (0.0, "")
        for i in range(a, b):
            g = (rows[i + 1][0] - max(r[1] for r in rows[max(a, i - 3):i + 1])) / 1000.0
            if g > 0:
                tot += g
                if g > best[0]:
                    best = (g, f"{short(rows[i][2])} -> {short(rows[i + 1][2])}")
        idle.append(tot)
        span.append((rows[b][1] - rows[a][1]) / 1000.0)
        big[best[1]] += 1
        busy.append(best[0])
    print(f"decode steps {len(idle)}: step {statistics.median(span):.1f} us median; idle "
          f"{statistics.median(idle):.1f} us median (p90 {sorted(idle)[9 * len(idle) // 10]:.1f}); "
          f"largest single gap {statistics.median(busy):.1f} us median")
    for k, v in big.most_common(5):
        print(f"  largest gap at: {k}  ({v} steps)")


if __name__ == "__main__":
    main()
