"""Loader / consumer ring GEMM (csrc/kernels/rgemm.hip) vs hipBLASLt at M = 256 on decode
projection shapes, cold weights (three copies rotate); us per call and the max error against
an fp32 reference.

    python tools/rgemm_probe.py
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner as gt  # noqa: E402

SHAPES = [("llama8b gate_up", 28672, 4096), ("llama8b qkv", 6144, 4096), ("llama8b o", 4096, 4096),
          ("70b-tp8 gate_up", 7168, 8192), ("qwen3 gate_up", 6144, 1024), ("qwen3 qkv", 4096, 1024)]


def main():
    ops.load_native(required=True)
    dev = "cuda"
    M = int(os.environ.get("RG_M", "256"))
    for name, N, K in SHAPES:
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(3)]
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = (x.float() @ ws[0].float().t())
        res = {"hipblaslt": gt._timed(lambda i: torch.nn.functional.linear(x, ws[i % 3]), 3)}
        errs = {}
        for bn in (64, 128):
            if N % bn:
                continue
            ops.rgemm(x, ws[0], out=y, bn=bn)
            torch.cuda.synchronize()
            errs[bn] = float((y.float() - ref).abs().max())
            res[f"rgemm{bn}"] = gt._timed(lambda i, bn=bn: ops.rgemm(x, ws[i % 3], out=y, bn=bn), 3)
        print(f"{name:16s} N={N:6d} K={K:5d} M={M}: " +
              " | ".join(f"{k} {v:7.1f}" for k, v in res.items()) +
              f"  max err {errs}  ring err flag {ops.rgemm_error(dev)}", flush=True)


if __name__ == "__main__":
    main()
