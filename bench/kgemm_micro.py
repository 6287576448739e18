"""Narrow-output decode GEMMs (O / down projections, N = d_model) on cold weights: the tuned
split-K decode GEMM + reduce (dgemm / gdgemm) vs the in-workgroup split-K kernel (kgemm.hip),
with the residual/next-norm epilogue the fused decode chain uses.

python bench/kgemm_micro.py [--model qwen3-0.6b]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops.gemm_tuner import _timed  # noqa: E402

SHAPES = {"qwen3-0.6b": (28, 1024, [("w_o", 2048), ("w_down", 3072)]),
          "llama-3-8b": (32, 4096, [("w_o", 4096), ("w_down", 14336)])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-0.6b")
    a = ap.parse_args()
    ops.load_native(required=True)
    L, N, projs = SHAPES[a.model]
    dev = "cuda"
    for name, K in projs:
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
        for M in (16, 64, 128, 256):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            res = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
            a_o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ss = torch.zeros(M, device=dev)
            ln = torch.ones(N, device=dev, dtype=torch.bfloat16)
            out = {}
            for s in (1, 2, 4, 8):
                for pf in (2, 4):
                    if not ops.dgemm_supported(M, N, K, s, pf, ops.EPI_RESNORM) or \
                            (s > 1 and K // s < 256):
                        continue
                    out[f"dgemm s{s}p{pf}"] = _timed(lambda i, s=s, pf=pf: ops.dgemm(
                        x, ws[i % L], splitk=s, pf=pf, out=res, epi=1, ss_out=ss, a_out=a_o,
                        ln_out=ln), L)
            for km in (16, 32):
                out[f"kgemm k{km}"] = _timed(lambda i, km=km: ops.dgemm(
                    x, ws[i % L], out=res, epi=1, ss_out=ss, a_out=a_o, ln_out=ln, km=km), L)
            best = min((v, k) for k, v in out.items() if k.startswith("dgemm"))
            bk = min((v, k) for k, v in out.items() if k.startswith("kgemm"))
            print(f"{a.model} {name} M={M:3d} N={N} K={K}: best split-K {best[1]} {best[0]:.1f} us"
                  f" | {bk[1]} {bk[0]:.1f} us | all: " +
                  " ".join(f"{k}={v:.1f}" for k, v in out.items()), flush=True)


if __name__ == "__main__":
    main()
