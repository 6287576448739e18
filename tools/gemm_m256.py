"""Decode-GEMM sweep at M = 256 (Llama-3-8B, Llama-3-70B TP=8 rank shard, Qwen3-0.6B): the
256-row LDS-DMA tiles (gdgemm bm=256, 8 waves) against hipBLASLt and the previous best
variants, on cold weights (a ring of distinct weight copies > the 256 MB Infinity Cache).
Every 256-row variant is checked against an fp32 reference before it is timed.

    python tools/gemm_m256.py [--M 256] [--only llama8b]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner as gt  # noqa: E402

SHAPES = {
    "llama8b": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096),
                ("down", 4096, 14336)],
    "llama70b_tp8": [("qkv", 1280, 8192), ("o", 8192, 1024), ("gate_up", 7168, 8192),
                     ("down", 8192, 3584)],
    "qwen3": [("qkv", 4096, 1024), ("o", 1024, 2048), ("gate_up", 6144, 1024),
              ("down", 1024, 3072)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=256)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    ops.load_native(required=True)
    M = a.M
    dev = "cuda"
    for model, shapes in SHAPES.items():
        if a.only and model != a.only:
            continue
        tot_best, tot_blas = 0.0, 0.0
        for name, N, K in shapes:
            nbytes = N * K * 2
            L = max(2, min(32, (600 << 20) // nbytes + 1))  # > Infinity Cache in flight
            ws_ = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16) * 0.5
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ref = (x.float() @ ws_[0].float().T)
            t_blas = gt._timed(lambda i: torch.nn.functional.linear(x, ws_[i % L]), L)
            res = [("hipblaslt", t_blas)]
            for s in (1, 2, 4, 8):
                if K % (64 * s) or K // s < 256:
                    continue
                for bn in (64, 128):
                    for bm in (128, 256):
                        if bm == 128 and bn != 128:
                            continue
                        for inl in ((False, True) if s > 1 else (False,)):
                            if not ops.dgemm_supported(M, N, K, s, 1, bn=bn, inlaunch=inl, bm=bm):
                                continue
                            for ns in ((3, 6) if bm == 256 and bn == 128 else
                                       (3,) if bm == 256 else (4,)):
                                fn = gt._gd_call(M, N, K, s, bn, ns, inl, y, x, ws_, 0, None,
                                                 None, None, None, bm)
                                if bm == 256:
                                    y.fill_(float("nan"))
                                    fn(0)
                                    torch.cuda.synchronize()
                                    err = (y.float() - ref).abs().max().item()
                                    scale = ref.abs().max().item()
                                    assert err <= 2e-2 * scale + 1e-2, (name, s, bn, ns, inl, err,
                                                                        scale)
                                t = gt._timed(fn, L)
                                res.append((f"s{s} g{bn}x{bm}" + ("d" if ns == 6 else "") +
                                            ("i" if inl else ""), t))
            res.sort(key=lambda r: r[1])
            best = res[0]
            tot_best += best[1]
            tot_blas += t_blas
            flops = 2.0 * M * N * K
            print(f"{model:13s} {name:8s} N={N:6d} K={K:6d}: best {best[0]:14s} {best[1]:7.1f} us "
                  f"({flops / best[1] / 1e6:6.0f} TFLOP/s, {nbytes / best[1] / 1e6:5.2f} TB/s "
                  f"weights) | hipBLASLt {t_blas:6.1f} | " +
                  "  ".join(f"{n} {t:.1f}" for n, t in res[1:8]), flush=True)
            del ws_
            torch.cuda.empty_cache()
        print(f"{model}: sum of best {tot_best:.1f} us/layer (hipBLASLt {tot_blas:.1f})",
              flush=True)


if __name__ == "__main__":
    main()
