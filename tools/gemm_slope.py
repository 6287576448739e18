"""Decode-GEMM cost model probe: time the K-split-in-workgroup kgemm (32 x 32 and 16 x 32
tiles, 256 workgroups at M = 256, N = 1024) and hipBLASLt over K, on cold (rotating, > the
Infinity Cache) and warm (one copy) weights, inside captured graphs.  The slope over K is the
per-CU ingress rate of the tile ((BM + 32) rows x K x 2 B per workgroup); the intercept is the
launch boundary + ramp + epilogue.

    python tools/gemm_slope.py
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
    M = 256
    for N in (1024, 4096):
        for K in (512, 1024, 2048, 4096, 8192):
            nbytes = N * K * 2
            L = max(2, min(64, (600 << 20) // nbytes + 1))
            ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16) * 0.5
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            row = []
            for tag, wl in (("cold", ws), ("warm", ws[:1])):
                n = len(wl) if tag == "cold" else 16
                t_b = gt._timed(lambda i: torch.nn.functional.linear(x, wl[i % len(wl)]), n)
                row.append(f"{tag}: blas {t_b:6.1f}")
                for km in (16, 32):
                    if not ops.kgemm_supported(M, N, K, km):
                        continue
                    t = gt._timed(lambda i, km=km: torch.ops.akap.kgemm(
                        y, x, wl[i % len(wl)], km, 0, 1e-6, None, None, None, None), n)
                    per_cu = (km + 32) * K * 2 / 1024
                    row.append(f"k{km} {t:6.1f} ({per_cu:5.0f} KB/WG)")
            print(f"N={N:5d} K={K:5d} | " + " | ".join(row), flush=True)
            del ws
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
