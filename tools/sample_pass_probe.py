"""Per-launch durations of the sampler's kernels at one batch size (for rocprofv3
--kernel-trace): B rows of bf16 [B, 151936] logits, one configuration launched back to back.

    rocprofv3 --kernel-trace --output-format csv -d /tmp/st -o run -- \
        python3 tools/sample_pass_probe.py --B 64 --k 50 --p 0.9
    python3 tools/sample_pass_probe.py --summarize /tmp/st/run_kernel_trace.csv
"""
from __future__ import annotations

import argparse
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def summarize(path: str) -> None:
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seq = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
            r.get("Grid_Size", "")) for r in rows if "sample" in r["Kernel_Name"]]
    # group by position inside a sample() call: chunk kernel starts a call
    calls, cur = [], []
    for name, us, grid in seq:
        if "chunk" in name and cur:
            calls.append(cur)
            cur = []
        cur.append((name, us, grid))
    if cur:
        calls.append(cur)
    by_pos = defaultdict(list)
    for c in calls[len(calls) // 4:]:  # skip warm-up calls
        for i, (name, us, grid) in enumerate(c):
            by_pos[(i, name.split("(")[0][-60:], grid)].append(us)
    for (i, name, grid), v in sorted(by_pos.items()):
        print(f"launch {i}: {sum(v) / len(v):8.1f} us  (n={len(v)}, grid {grid})  {name}")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--k", type=int, default=50)
    ap.add_argument("--p", type=float, default=0.9)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--summarize", default="")
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize)
        return
    import torch

    from aws_k8s_ansible_provisioner_amd import ops

    ops.load_native(required=True)
    dev, V, B = "cuda", 151936, a.B
    x = (torch.randn(B, V, device=dev) * 3).to(torch.bfloat16)
    temp = torch.ones(B, device=dev)
    tk = torch.full((B,), a.k, device=dev, dtype=torch.int32)
    tp = torch.full((B,), a.p, device=dev)
    seeds = torch.arange(B, device=dev, dtype=torch.int64)
    steps = torch.zeros(B, device=dev, dtype=torch.int32)
    for _ in range(a.iters):
        ops.sample(x, temp, tk, tp, seeds, steps, filtered=True)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
