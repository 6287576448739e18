"""Grouped expert GEMMs of a Mixtral-8x7B decode layer, cold weights: the 64x64 moe_gemm
(+ separate silu_and_mul) vs the 32x128 k-pipelined moe_dgemm (SwiGLU epilogue).

python bench/moe_gemm_micro.py [--T 128] [--layers 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402


def timed(fn, n, reps=3):
    fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / (reps * n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=128)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--E", type=int, default=8)
    ap.add_argument("--d", type=int, default=4096)
    ap.add_argument("--F", type=int, default=14336)
    a = ap.parse_args()
    ops.load_native(required=True)
    dev = "cuda"
    T, E, d, F, K = a.T, a.E, a.d, a.F, 2
    L = a.layers
    w13 = [torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
    w2 = [torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
    h = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    logits = torch.randn(T, E, device=dev, dtype=torch.bfloat16)
    tw, ids = ops.moe_topk_softmax(logits, K)
    n = T * K
    gb13 = E * 2 * F * d * 2 / 1e9
    gb2 = E * d * F * 2 / 1e9
    for blk, name in ((64, "moe_gemm 64x64"), (32, "moe_dgemm 32x128"), (64, "moe_dgemm 64x128")):
        cap = ops.moe_capacity(n, E, blk)
        tiles = cap // blk
        inv = torch.empty(n, dtype=torch.int32, device=dev)
        te = torch.empty(tiles, dtype=torch.int32, device=dev)
        sid, off, npad = ops.moe_align(ids, E, blk, inv=inv, tile_expert=te)
        used = int((te >= 0).sum())
        if name.startswith("moe_gemm"):
            y1 = torch.empty(cap, 2 * F, device=dev, dtype=torch.bfloat16)
            act = torch.empty(cap, F, device=dev, dtype=torch.bfloat16)
            y2 = torch.empty(cap, d, device=dev, dtype=torch.bfloat16)
            t13 = timed(lambda i: (torch.ops.akap.moe_gemm(y1, h, w13[i % L], sid, te, n, K, True),
                                   torch.ops.akap.silu_and_mul(act, y1)), L)
            t2 = timed(lambda i: torch.ops.akap.moe_gemm(y2, act, w2[i % L], sid, te, n, K, False), L)
        else:
            act = torch.empty(cap, F, device=dev, dtype=torch.bfloat16)
            y2 = torch.empty(cap, d, device=dev, dtype=torch.bfloat16)
            t13 = timed(lambda i: torch.ops.akap.moe_dgemm(act, h, w13[i % L], sid, te, n, K, True,
                                                           True, 4, blk), L)
            t2 = timed(lambda i: torch.ops.akap.moe_dgemm(y2, act, w2[i % L], sid, te, n, K, False,
                                                          False, 4, blk), L)
        extra = ""
        if name.startswith("moe_dgemm"):
            out = torch.empty(T, d, device=dev, dtype=torch.bfloat16)
            tc = timed(lambda i: torch.ops.akap.moe_combine(y2, tw, inv, out), L)
            extra = f"  w2+combine {t2 + tc:6.1f}"
            for S in (2, 4, 8):
                pf = 4 if (F // S) % 256 == 0 else 2
                P = torch.empty(S * cap * d, device=dev, dtype=torch.float32)
                ts = timed(lambda i, S=S, P=P, pf=pf: (
                    torch.ops.akap.moe_dgemm(P, act, w2[i % L], sid, te, n, K, False, False, pf,
                                             blk, S),
                    torch.ops.akap.moe_combine_split(P, tw, inv, out, S, cap)), L)
                extra += f"  split{S} {ts:6.1f}"
        print(f"T={T} {name:18s} tiles used {used:3d}/{tiles}: w13(+silu) {t13:7.1f} us "
              f"({gb13 / t13 * 1e3:.2f} TB/s)  w2 {t2:7.1f} us ({gb2 / t2 * 1e3:.2f} TB/s)" + extra,
              flush=True)


if __name__ == "__main__":
    main()
