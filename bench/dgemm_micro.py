"""Fused decode GEMM (csrc/kernels/dgemm.hip) vs the unfused decode-layer sequence, cold weights.

For each projection of a decode layer the baseline is what the engine runs today:
  qkv / gate_up : fused_add_rms_norm kernel + hipBLASLt GEMM
  o             : hipBLASLt GEMM
  down          : silu_and_mul kernel + hipBLASLt GEMM
and the candidate is ONE dgemm launch (prologue folded into the operand staging) at each
(split-K, prefetch depth).  Every timing rotates through enough distinct weight copies
(>= 1 GiB) inside one captured hipGraph that each call reads its weights cold, as in a
decode step.  Also checks every candidate's output against the baseline.

    python bench/dgemm_micro.py [--model qwen3-0.6b|llama-3-8b] [--m 64,128,256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402

MODELS = {  # d, q+2kv rows, q cols, ffn
    "qwen3-0.6b": (1024, 4096, 2048, 3072),
    "llama-3-8b": (4096, 6144, 4096, 14336),
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
    ap.add_argument("--splits", default="1,2,4,8")
    ap.add_argument("--pfs", default="1,2,4")
    a = ap.parse_args()
    ops.load_native(required=True)
    d, nqkv, dq, ffn = MODELS[a.model]
    eps = 1e-6
    projs = {  # name: (N, K, prologue)
        "qkv": (nqkv, d, ops.PRO_ADDNORM),
        "o": (d, dq, ops.PRO_PLAIN),
        "gate_up": (2 * ffn, d, ops.PRO_ADDNORM),
        "down": (d, ffn, ops.PRO_SILU),
    }
    dev = "cuda"
    for M in [int(m) for m in a.m.split(",")]:
        for name, (N, K, pro) in projs.items():
            wbytes = N * K * 2
            copies = max(2, (1 << 30) // wbytes + 1)
            ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
            ln = torch.rand(K, device=dev, dtype=torch.bfloat16) + 0.5
            xin = torch.randn(M, 2 * K if pro == ops.PRO_SILU else K, device=dev,
                              dtype=torch.bfloat16)
            res = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            res_base = res.clone()
            rout = torch.empty_like(res)
            h = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            iters = max(copies, 8)

            def base(i):
                if pro == ops.PRO_ADDNORM:
                    torch.ops.akap.fused_add_rmsnorm(h, res_base, xin, ln, eps)
                    a_ = h
                elif pro == ops.PRO_SILU:
                    torch.ops.akap.silu_and_mul(h, xin)
                    a_ = h
                else:
                    a_ = xin
                return torch.nn.functional.linear(a_, ws[i % copies])

            t_base = timed(base, iters)
            # reference output (fresh residual: the timed base() accumulated into res_base)
            res_base.copy_(res)
            y_ref = base(0).float()
            out = [f"base {t_base:6.1f}"]
            best = (t_base, "base")
            for s in [int(v) for v in a.splits.split(",")]:
                for pf in [int(v) for v in a.pfs.split(",")]:
                    if not ops.dgemm_supported(M, N, K, s, pf):
                        continue
                    wsp = torch.empty(max(1, s * M * N + s * M), device=dev, dtype=torch.float32)

                    def cand(i, s=s, pf=pf, wsp=wsp):
                        torch.ops.akap.dgemm(y, xin, ws[i % copies], wsp, pro, s, pf, res, rout,
                                             ln, eps)

                    t = timed(cand, iters)
                    cand(0)
                    torch.cuda.synchronize()
                    err = (y.float() - y_ref).abs().max().item() / (y_ref.abs().max().item() + 1e-6)
                    flag = "" if err < 2e-2 else f"!ERR{err:.3f}"
                    out.append(f"s{s}p{pf} {t:6.1f}{flag}")
                    if t < best[0] and not flag:
                        best = (t, f"s{s}p{pf}")
            print(f"M={M:4d} {name:8s} N={N:6d} K={K:6d}: " + " ".join(out) +
                  f"   -> best {best[1]} {best[0]:.1f} us ({t_base / best[0]:.2f}x)", flush=True)
            if pro != ops.PRO_PLAIN:  # what the prologue costs: same shape, plain operand
                xp = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
                outp = [f"blaslt {timed(lambda i: torch.nn.functional.linear(xp, ws[i % copies]), iters):6.1f}"]
                for s in [int(v) for v in a.splits.split(",")]:
                    for pf in [int(v) for v in a.pfs.split(",")]:
                        if not ops.dgemm_supported(M, N, K, s, pf):
                            continue
                        wsp = torch.empty(max(1, s * M * N), device=dev, dtype=torch.float32)
                        t = timed(lambda i, s=s, pf=pf, wsp=wsp: torch.ops.akap.dgemm(
                            y, xp, ws[i % copies], wsp, 0, s, pf), iters)
                        outp.append(f"s{s}p{pf} {t:6.1f}")
                print(f"        {'(plain)':8s} {'':25s}  " + " ".join(outp), flush=True)
            del ws


if __name__ == "__main__":
    main()
