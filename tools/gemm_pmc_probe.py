"""One decode GEMM variant launched back to back on cold weights, for rocprofv3 --pmc passes
(Llama-3-8B gate_up at M = 256 by default: the 256-row LDS-DMA tile, s1 g128x256).

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python3 tools/gemm_pmc_probe.py [--N 28672 --K 4096]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner as gt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=256)
    ap.add_argument("--N", type=int, default=28672)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--split", type=int, default=1)
    ap.add_argument("--bn", type=int, default=128)
    ap.add_argument("--bm", type=int, default=256)
    ap.add_argument("--ns", type=int, default=3)
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    ops.load_native(required=True)
    M, N, K = a.M, a.N, a.K
    L = max(2, min(32, (600 << 20) // (N * K * 2) + 1))
    ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(L)]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16) * 0.5
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    fn = gt._gd_call(M, N, K, a.split, a.bn, a.ns, False, y, x, ws, 0, None, None, None, None,
                     a.bm)
    for i in range(a.iters):
        fn(i)
    torch.cuda.synchronize()
    t = gt._timed(fn, L)
    print(f"M={M} N={N} K={K} s{a.split} g{a.bn}x{a.bm} ns={a.ns}: {t:.1f} us", flush=True)


if __name__ == "__main__":
    main()
