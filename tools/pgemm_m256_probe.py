"""How fast is the 256 x 256 pgemm tile body at decode batch M = 256 (one row tile)?  Llama-3-8B
projections on cold weights (rotating copies > the Infinity Cache), pgemm (no split: N/256
workgroups) vs hipBLASLt, in captured graphs.  Tells whether a split-K / stream-K launcher
over this body can beat the decode GEMMs (tools/gemm_m256.py)."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner as gt  # noqa: E402

SHAPES = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096),
          ("down", 4096, 14336), ("70b-tp8 gate_up", 7168, 8192)]


def main():
    ops.load_native(required=True)
    dev = "cuda"
    M = 256
    for name, N, K in SHAPES:
        L = max(2, min(32, (600 << 20) // (N * K * 2) + 1))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t_b = gt._timed(lambda i: torch.nn.functional.linear(x, ws[i % L]), L)
        t_p = gt._timed(lambda i: torch.ops.akap.pgemm(y, x, ws[i % L], 0, None), L)
        fl = 2.0 * M * N * K
        ref = x.float() @ ws[0].float().t()
        sk = []
        for s in range(2, 33):
            if not ops.dgemm_supported(M, N, K, s, 1, 0, bn=256, inlaunch=True, bm=256):
                continue
            if s not in (2, 3, 4, 5, 6, 8, 10, 12, 14, 16, 20, 24, 28, 32):
                continue
            ops.dgemm(x, ws[0], splitk=s, bn=256, bm=256, inlaunch=True, out=y)
            torch.cuda.synchronize()
            err = (y.float() - ref).abs().max().item() / ref.abs().max().item()
            assert err < 2e-2, (name, s, err)
            t = gt._timed(lambda i, s=s: ops.dgemm(x, ws[i % L], splitk=s, bn=256, bm=256,
                                                   inlaunch=True, out=y), L)
            sk.append((t, s))
        sk.sort()
        print(f"{name:16s} N={N:6d} K={K:6d}: hipBLASLt {t_b:6.1f} us ({fl / t_b / 1e6:5.0f} TF) | "
              f"pgemm {N // 256:4d} WGs {t_p:6.1f} us ({fl / t_p / 1e6:5.0f} TF, "
              f"{fl / t_p / 1e6 * 256 / (N // 256):5.0f} TF per-CU-scaled) | split-K in-launch: " +
              "  ".join(f"s{s} {t:.1f}" for t, s in sk[:6]), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
