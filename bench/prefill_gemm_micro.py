"""Prefill GEMM shapes: hipBLASLt (torch) TFLOP/s, and the hand-written prefill GEMM when
built (torch.ops.akap.pgemm), on random operands, median of interleaved rounds.

python bench/prefill_gemm_micro.py [--M 16384]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402

SHAPES = {
    "qwen3-0.6b": [("qkv", 4096, 1024), ("o", 1024, 2048), ("gate_up", 6144, 1024),
                   ("down", 1024, 3072)],
    "llama-3-8b": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096),
                   ("down", 4096, 14336)],
}


def bench(fns, rounds=5, iters=10):
    res = {k: [] for k in fns}
    for _ in range(rounds):
        for k, f in fns.items():
            f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            for _ in range(iters):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1000 / iters)
    return {k: statistics.median(v) for k, v in res.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=16384)
    a = ap.parse_args()
    ops.load_native(required=True)
    has_pgemm = hasattr(torch.ops.akap, "pgemm")
    for model, shapes in SHAPES.items():
        for name, N, K in shapes:
            M = a.M
            x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
            w = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            fns = {"hipblaslt": lambda: torch.nn.functional.linear(x, w)}
            if has_pgemm:
                fns["pgemm"] = lambda: torch.ops.akap.pgemm(y, x, w)
            t = bench(fns)
            fl = 2.0 * M * N * K
            line = f"{model:11s} {name:8s} M={M} N={N:6d} K={K:6d}: " + "  ".join(
                f"{k} {v:8.1f} us {fl / v / 1e6:7.1f} TF" for k, v in t.items())
            if has_pgemm:
                ref = torch.nn.functional.linear(x, w).float()
                torch.ops.akap.pgemm(y, x, w)
                line += f"  max rel err {((y.float() - ref).abs().max() / ref.abs().max()).item():.2e}"
            print(line, flush=True)
            del x, w, y


if __name__ == "__main__":
    main()
