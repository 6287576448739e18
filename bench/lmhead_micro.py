"""Decode LM-head GEMM micro-benchmark: hipBLASLt vs the wide-row kernel (wgemm.hip) vs the
64-row LDS-DMA decode GEMM (gdgemm.hip), cold weights (> 256 MB Infinity Cache per call).

python bench/lmhead_micro.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops.gemm_tuner import _timed  # noqa: E402


def main():
    ops.load_native(required=True)
    dev = "cuda"
    for name, V, K in (("qwen3-0.6b", 151936, 1024), ("llama-3-8b", 128256, 4096)):
        w = torch.randn(V, K, device=dev, dtype=torch.bfloat16) * 0.02
        wb = V * K * 2
        for M in (16, 64, 128, 256):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            y = torch.empty(M, V, device=dev, dtype=torch.bfloat16)
            res = {}
            res["hipblaslt"] = _timed(lambda i: torch.nn.functional.linear(x, w), 4)
            res["wgemm"] = _timed(lambda i: torch.ops.akap.wgemm(y, x, w), 4)
            ws = torch.empty(1, device=dev, dtype=torch.float32)
            res["gdgemm128"] = _timed(lambda i: torch.ops.akap.dgemm(
                y, x, w, ws, 0, 1, 1, None, None, None, 1e-6, 0, None, None, None, None, 128, 0,
                None), 4)
            ref = (x.float() @ w.float().T)
            torch.ops.akap.wgemm(y, x, w)
            err = (y.float() - ref).abs().max().item()
            print(f"{name} M={M:4d} V={V} K={K}: " + "  ".join(
                f"{k} {v:7.1f} us ({wb / v / 1e6:4.2f} TB/s)" for k, v in res.items()) +
                f"  wgemm max err {err:.3g}", flush=True)
        del w


if __name__ == "__main__":
    main()
