"""Decode GEMMs, cold weights: hipBLASLt vs the register-ring dgemm vs the LDS-DMA ring
(gdgemm.hip, 64x64 / 64x128 tiles), plain store epilogue.
python bench/gdgemm_micro.py [--model qwen3-0.6b|llama-3-8b] [--m 64,128,256]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402

SHAPES = {
    "qwen3-0.6b": {"qkv": (4096, 1024), "o": (1024, 2048), "gate_up": (6144, 1024),
                   "down": (1024, 3072)},
    "llama-3-8b": {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
                   "down": (4096, 14336)},
}


def timed(fn, iters):
    fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(iters):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    g.replay()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / (2 * iters)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-0.6b")
    ap.add_argument("--m", default="64,128,256")
    a = ap.parse_args()
    ops.load_native(required=True)
    for M in [int(v) for v in a.m.split(",")]:
        for name, (N, K) in SHAPES[a.model].items():
            copies = max(2, (1 << 30) // (N * K * 2) + 1)
            ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
                  for _ in range(copies)]
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            n = max(copies, 8)
            res = [f"blaslt {timed(lambda i: torch.nn.functional.linear(x, ws[i % copies]), n):6.1f}"]
            best_reg = None
            for s in (1, 2, 4, 8):
                for pf in (2, 4):
                    if not ops.dgemm_supported(M, N, K, s, pf) or (s > 1 and K // s < 256):
                        continue
                    wsp = torch.empty(max(1, s * M * N), device="cuda", dtype=torch.float32)
                    t = timed(lambda i, s=s, pf=pf, wsp=wsp: torch.ops.akap.dgemm(
                        y, x, ws[i % copies], wsp, 0, s, pf), n)
                    if best_reg is None or t < best_reg[0]:
                        best_reg = (t, f"s{s}p{pf}")
            res.append(f"dgemm {best_reg[0]:6.1f} ({best_reg[1]})")
            for bn in (64, 128):
                for s in (1, 2, 4, 8):
                    if not ops.dgemm_supported(M, N, K, s, 1, bn=bn):
                        continue
                    wsp = torch.empty(max(1, s * M * N), device="cuda", dtype=torch.float32)
                    t = timed(lambda i, s=s, bn=bn, wsp=wsp: torch.ops.akap.dgemm(
                        y, x, ws[i % copies], wsp, 0, s, 1, None, None, None, 1e-6, 0, None,
                        None, None, None, bn), n)
                    res.append(f"g{bn}s{s} {t:6.1f}")
            # correctness of the last variant
            ref_ = x.float() @ ws[0].float().t()
            wsp = torch.empty(1, device="cuda", dtype=torch.float32)
            torch.ops.akap.dgemm(y, x, ws[0], wsp, 0, 1, 1, None, None, None, 1e-6, 0, None,
                                 None, None, None, 128)
            err = (y.float() - ref_).abs().max().item() / ref_.abs().max().item()
            print(f"M={M:4d} {name:8s} N={N:6d} K={K:6d}: " + "  ".join(res) +
                  (f"  !ERR {err:.3f}" if err > 2e-2 else ""), flush=True)
            del ws


if __name__ == "__main__":
    main()
