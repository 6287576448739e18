"""One prefill GEMM launched back to back, for rocprofv3 --pmc / --kernel-trace passes:
the hand-written pgemm (csrc/kernels/pgemm.hip) or, with --lib, hipBLASLt on the same shape.

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python3 tools/pgemm_pmc_probe.py [--lib] [--M --N --K]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=8192)
    ap.add_argument("--N", type=int, default=6144)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--lib", action="store_true")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    ops.load_native(required=True)
    x = torch.randn(a.M, a.K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(a.N, a.K, device="cuda", dtype=torch.bfloat16) * 0.02
    y = torch.empty(a.M, a.N, device="cuda", dtype=torch.bfloat16)
    fn = (lambda: torch.matmul(x, w.t(), out=y)) if a.lib else (lambda: ops.pgemm(x, w, out=y))
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / a.iters
    print(f"{'hipBLASLt' if a.lib else 'pgemm'} M={a.M} N={a.N} K={a.K}: {t * 1e3:.1f} us "
          f"= {2 * a.M * a.N * a.K / t / 1e9:.0f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
