#!/usr/bin/env python3
"""What a persistent decode layer could save at most: the GPU-idle time at each kernel boundary
of the steady decode step, measured from a rocprofv3 --kernel-trace CSV (round 6, VERDICT r5
item 1 step B).

For every pair of consecutive dispatches inside decode graph replays (the dispatches between
two greedy-sampling launches that contain no prefill-attention launch), the boundary is
start(next) - end(prev) on the GPU clock.  Reported per (prev kernel -> next kernel) pair:
count, mean and median idle us, plus the per-step total of the GEMM-chain boundaries (the ones a
persistent O -> gate_up -> down launch would remove) and each kernel's mean duration.

    python tools/decode_boundaries.py run_kernel_trace.csv [--min-steps 50]
"""
import csv
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0].replace("void ", "").replace("akap::", "")
    for k in ("paged_attn_decode", "kgemm_kernel", "gdgemm_kernel", "dgemm_kernel", "wgemm_kernel",
              "argmax", "sample_kernel", "embedding_prep", "h2d_stage", "rmsnorm", "qk_norm_rope"):
        if k in n:
            return n if "<" in n and k in ("kgemm_kernel", "gdgemm_kernel", "dgemm_kernel") else k
    return n[:40]


def main() -> int:
    path = sys.argv[1]
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # split into steps at each sampling launch (argmax / sample_kernel ends a step)
    steps, cur = [], []
    for r in rows:
        cur.append(r)
        if "argmax_kernel" in r[2] or "sample_kernel" in r[2]:
            steps.append(cur)
            cur = []
    dec = [s for s in steps if not any("prefill" in r[2] for r in s)
           and sum("paged_attn_decode" in r[2] for r in s) >= 16]
    # keep the steady full-batch steps: the most common step length
    lens = defaultdict(int)
    for s in dec:
        lens[len(s)] += 1
    L = max(lens, key=lens.get)
    dec = [s for s in dec if len(s) == L]
    gaps = defaultdict(list)
    durs = defaultdict(list)
    step_us = []
    for s in dec:
        step_us.append((s[-1][1] - s[0][0]) / 1e3)
        for a, b in zip(s, s[1:]):
            gaps[(short(a[2]), short(b[2]))].append((b[0] - a[1]) / 1e3)
        for r in s:
            durs[short(r[2])].append((r[1] - r[0]) / 1e3)
    print(f"# decode boundaries: {len(dec)} steady decode steps of {L} dispatches "
          f"(median step {statistics.median(step_us):.1f} us, first dispatch start to sampling end)")
    print()
    print("| prev -> next | per step | mean idle us | median idle us |")
    print("|---|---:|---:|---:|")
    tot = 0.0
    for (a, b), v in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
        per = len(v) / len(dec)
        tot += statistics.mean(v) * per
        print(f"| `{a}` -> `{b}` | {per:.0f} | {statistics.mean(v):.2f} | {statistics.median(v):.2f} |")
    print()
    print(f"total idle per step: {tot:.1f} us")
    print()
    # idle at each step's start (previous step's sampling end -> this step's first dispatch)
    # plus inside its first 4 dispatches (the host-launched staging / gather before the graph)
    head = []
    for a_, b_ in zip(dec, dec[1:]):
        head.append(sum(max(0, y[0] - x[1]) for x, y in zip([a_[-1]] + b_[:4], b_[:5])) / 1e3)
    if head:
        hs = sorted(head)
        pct = lambda q: hs[min(len(hs) - 1, int(q * len(hs)))]
        print(f"step-start idle per step (us): p50 {pct(0.5):.1f}  p90 {pct(0.9):.1f}  "
              f"p99 {pct(0.99):.1f}  max {hs[-1]:.1f}  mean {statistics.mean(hs):.1f}  "
              f"steps over 100 us: {sum(h > 100 for h in hs)} of {len(hs)}")
        print()
    print("| kernel | per step | mean us |")
    print("|---|---:|---:|")
    for k, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        print(f"| `{k}` | {len(v) / len(dec):.0f} | {statistics.mean(v):.2f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
