"""Sampler microbench (csrc/kernels/sampling.hip) at decode batch sizes on Qwen3's vocab:
greedy, T=1.0, top-k 50, top-p 0.9 and top-k + top-p, bf16 logits [B, 151936], timed as a
captured graph of back-to-back launches.  The memory floor is B * V * 2 bytes at ~6 TB/s.

    python tools/sample_bench.py
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner as gt  # noqa: E402


def main():
    ops.load_native(required=True)
    dev = "cuda"
    V = 151936
    for B in (1, 16, 64, 256):
        x = (torch.randn(B, V, device=dev) * 3).to(torch.bfloat16)
        # unit-scale logits: top-p 0.9's threshold lies far below the 256-key window under the
        # max, so these rows take the distributed histogram passes (the fallback)
        xf = torch.randn(B, V, device=dev).to(torch.bfloat16)
        seeds = torch.arange(B, device=dev, dtype=torch.int64)
        steps = torch.zeros(B, device=dev, dtype=torch.int32)
        tok = torch.empty(B, dtype=torch.int64, device=dev)
        lp = torch.empty(B, dtype=torch.float32, device=dev)
        cases = {
            "greedy": (0.0, 0, 1.0),
            "T=1.0": (1.0, 0, 1.0),
            "top-k 50": (1.0, 50, 1.0),
            "top-p 0.9": (1.0, 0, 0.9),
            "k50+p0.9": (1.0, 50, 0.9),
            "top-p 0.9 flat": (1.0, 0, 0.9),
        }
        row = []
        for name, (t, k, p) in cases.items():
            temp = torch.full((B,), t, device=dev)
            tk = torch.full((B,), k, device=dev, dtype=torch.int32)
            tp = torch.full((B,), p, device=dev)
            filt = k > 0 or p < 1.0  # the engine skips the threshold passes otherwise
            xx = xf if name.endswith("flat") else x
            us = gt._timed(lambda i: ops.sample(xx, temp, tk, tp, seeds, steps, tok, lp,
                                                filtered=filt), 20)
            row.append(f"{name} {us:7.1f}")
        floor = B * V * 2 / 6.0e6
        print(f"B={B:4d} (read floor {floor:5.1f} us): " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
