"""Prefill attention microbenchmark: 64-row per-wave kernel vs 128-row flash-style kernel.

python bench/prefill_attn_micro.py [--B 32] [--L 512] [--hq 16 --hkv 8]"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--hq", type=int, default=16)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    ops.load_native(required=True)
    dev, D, BS = "cuda", 128, 32
    B, L, G = a.B, a.L, a.hq // a.hkv
    nbp = math.ceil(L / BS)
    NB = B * nbp + 4
    kc = torch.randn(NB, a.hkv, BS, D, dtype=torch.bfloat16, device=dev)
    vc = torch.randn(NB, a.hkv, BS // 8, D, 8, dtype=torch.bfloat16, device=dev)
    perm = torch.randperm(NB)
    bt = torch.zeros(B, 4096 // BS, dtype=torch.int32)
    for s in range(B):
        bt[s, :nbp] = perm[s * nbp:(s + 1) * nbp].to(torch.int32)
    q = torch.randn(B * L, a.hq, D, dtype=torch.bfloat16, device=dev)
    out = torch.empty_like(q)
    sl = torch.full((B,), L, dtype=torch.int32, device=dev)
    qs = torch.arange(0, B * L + 1, L, dtype=torch.int32, device=dev)
    flops = B * a.hq * L * L / 2 * D * 4
    for rows in (64, 128, 256):
        ts, tr = [], []
        for s in range(B):
            for r in range(0, L * G, rows):
                ts.append(s)
                tr.append(r)
        ts = torch.tensor(ts, dtype=torch.int32, device=dev)
        tr = torch.tensor(tr, dtype=torch.int32, device=dev)
        f = lambda: ops.paged_attention_prefill(out, q, kc, vc, bt.to(dev), sl, qs, ts, tr, G,  # noqa
                                                1 / math.sqrt(D), tile_rows=rows)
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(a.iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / a.iters
        print(f"prefill B={B} L={L} hq={a.hq} hkv={a.hkv} tile_rows={rows:3d}: {us:8.1f} us "
              f"{flops / us / 1e6:7.1f} TFLOP/s (causal)", flush=True)


if __name__ == "__main__":
    main()
