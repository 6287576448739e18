"""Mixtral-8x7B MoE block at prefill sizes (TP=1): the device-side grouped path
(ops.fused_moe: moe_align + grouped MFMA GEMMs + combine, no host sync) against a per-expert
hipBLASLt loop driven by host-side counts (the round-2 path above 1024 tokens), and a
correctness check of the grouped path against an fp32 reference on a token subset.

    python tools/moe_prefill.py [--T 1024 4096 16384]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def loop_moe(h, w13, w2, w, ids, E, K):
    flat = ids.reshape(-1).long()
    order = torch.argsort(flat, stable=True)
    tok = order // K
    counts = torch.bincount(flat, minlength=E).tolist()
    x = h[tok]
    y = torch.empty_like(x)
    o = 0
    for j, c in enumerate(counts):
        if c:
            y[o:o + c] = F.linear(ops.silu_and_mul(F.linear(x[o:o + c], w13[j])), w2[j])
            o += c
    out = torch.zeros(h.shape, dtype=torch.float32, device=h.device)
    out.index_add_(0, tok, y.float() * w.reshape(-1)[order].float()[:, None])
    return out.to(h.dtype)


def grouped_moe(h, w13t, w2t, w, ids, E, K):
    """No host sync: rows sorted by expert on the device, torch._grouped_mm (the ROCm library
    grouped GEMM) over device-side group offsets, index_add combine."""
    flat = ids.reshape(-1).long()
    order = torch.argsort(flat, stable=True)
    tok = order // K
    offs = torch.cumsum(torch.bincount(flat, minlength=E), 0).to(torch.int32)
    x = h[tok]
    a = ops.silu_and_mul(torch._grouped_mm(x, w13t, offs=offs))
    y = torch._grouped_mm(a, w2t, offs=offs)
    out = torch.zeros(h.shape, dtype=torch.float32, device=h.device)
    out.index_add_(0, tok, y.float() * w.reshape(-1)[order].float()[:, None])
    return out.to(h.dtype)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, nargs="+", default=[1024, 4096, 16384])
    a = ap.parse_args()
    ops.load_native(required=True)
    E, K, d, Fn = 8, 2, 4096, 14336
    dev = "cuda"
    w13 = torch.randn(E, 2 * Fn, d, device=dev, dtype=torch.bfloat16) * 0.02
    w2 = torch.randn(E, d, Fn, device=dev, dtype=torch.bfloat16) * 0.02
    router = torch.randn(E, d, device=dev, dtype=torch.bfloat16) * 0.02
    for T in a.T:
        h = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
        w, ids = ops.moe_router_topk(h, router, K, renormalize=True)
        y = ops.fused_moe(h, w13, w2, w, ids)
        ref = loop_moe(h, w13, w2, w, ids, E, K)
        err = (y.float() - ref.float()).abs().max().item()
        scale = ref.float().abs().max().item()
        t_f = timed(lambda: ops.fused_moe(h, w13, w2, w, ids))
        t_l = timed(lambda: loop_moe(h, w13, w2, w, ids, E, K))
        flops = 2.0 * T * K * (2 * Fn * d + d * Fn)
        gm = ""
        try:
            w13t, w2t = w13.transpose(1, 2), w2.transpose(1, 2)
            yg = grouped_moe(h, w13t, w2t, w, ids, E, K)
            eg = (yg.float() - ref.float()).abs().max().item()
            t_g = timed(lambda: grouped_moe(h, w13t, w2t, w, ids, E, K))
            gm = f"  torch._grouped_mm {t_g:8.2f} ms ({flops / t_g / 1e9:6.0f} TFLOP/s, diff {eg:.4f})"
        except Exception as e:  # not supported on this build / layout
            gm = f"  torch._grouped_mm unavailable: {type(e).__name__}: {str(e)[:160]}"
        print(f"T={T:6d}: fused_moe {t_f:8.2f} ms ({flops / t_f / 1e9:6.0f} TFLOP/s)  "
              f"per-expert hipBLASLt loop {t_l:8.2f} ms ({flops / t_l / 1e9:6.0f} TFLOP/s)  "
              f"max|diff| {err:.4f} of {scale:.3f}" + gm, flush=True)
        assert err <= 3e-2 * scale + 1e-2


if __name__ == "__main__":
    main()
