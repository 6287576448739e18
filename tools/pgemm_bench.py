"""Microbench of the hand-written prefill GEMM (csrc/kernels/pgemm.hip) against the library
paths it would replace: hipBLASLt (torch.matmul) for the dense projections and
torch._grouped_mm for the expert-grouped MoE GEMMs.  Shapes are the prefill GEMMs of the
headline model (Qwen3-8B: qkv 6144x4096, o 4096x4096, gate_up 24576x4096, down 4096x12288),
Llama-3-8B's, and Mixtral-8x7B's grouped expert GEMMs at 16384 routed rows.

    python tools/pgemm_bench.py [--json gpurun_out/pgemm.json]
Prints one line per shape: TFLOP/s of each path and the ratio."""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402

DENSE = [  # (name, M, N, K)
    ("qwen3-8b qkv", 8192, 6144, 4096),
    ("qwen3-8b o", 8192, 4096, 4096),
    ("qwen3-8b gate_up", 8192, 24576, 4096),
    ("qwen3-8b down", 8192, 4096, 12288),
    ("llama3-8b gate_up", 8192, 28672, 4096),
    ("llama3-8b down", 8192, 4096, 14336),
    ("qkv M=2048", 2048, 6144, 4096),
    # the headline model's prefill projections at a 16384-token chunk (Qwen3-0.6B)
    ("qwen3-0.6b qkv", 16384, 4096, 1024),
    ("qwen3-0.6b o", 16384, 1024, 2048),
    ("qwen3-0.6b gate_up", 16384, 6144, 1024),
    ("qwen3-0.6b down", 16384, 1024, 3072),
    ("gate_up M=16384", 16384, 24576, 4096),
]
# every dense prefill projection of the two benchmark models at a
# 16384-token chunk (silu: the gate|up GEMM with the SwiGLU epilogue vs hipBLASLt +
# silu_and_mul), and Mixtral's grouped w13 (SwiGLU) / w2
VERDICT = [  # (name, M, N, K, silu)
    ("qwen3-0.6b qkv", 16384, 4096, 1024, False),
    ("qwen3-0.6b o", 16384, 1024, 2048, False),
    ("qwen3-0.6b gate_up", 16384, 6144, 1024, False),
    ("qwen3-0.6b gate_up silu", 16384, 6144, 1024, True),
    ("qwen3-0.6b down", 16384, 1024, 3072, False),
    ("llama3-8b qkv", 16384, 6144, 4096, False),
    ("llama3-8b o", 16384, 4096, 4096, False),
    ("llama3-8b gate_up", 16384, 28672, 4096, False),
    ("llama3-8b gate_up silu", 16384, 28672, 4096, True),
    ("llama3-8b down", 16384, 4096, 14336, False),
]
GROUPED = [  # (name, rows, experts, N, K)
    ("mixtral w13", 16384 * 2, 8, 28672, 4096),
    ("mixtral w2", 16384 * 2, 8, 4096, 14336),
    ("qwen3-moe w13 128e", 16384 * 8, 128, 1536, 2048),
    ("qwen3-moe w2 128e", 16384 * 8, 128, 2048, 768),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters / 1e3


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="")
    ap.add_argument("--set", default="all", choices=["all", "verdict"])
    a = ap.parse_args()
    dev = "cuda"
    rows = []
    if a.set == "verdict":
        for name, M, N, K, silu in VERDICT:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            fl = 2.0 * M * N * K
            if silu:
                act = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
                t_lib = timeit(lambda: ops.silu_and_mul(torch.matmul(x, w.t(), out=y), act))
                t_pg = timeit(lambda: ops.pgemm(x, w, silu=True, out=act))
                ref = ops.silu_and_mul(torch.matmul(x, w.t()))
                err = (ops.pgemm(x, w, silu=True).float() - ref.float()).abs().max().item()
            else:
                t_lib = timeit(lambda: torch.matmul(x, w.t(), out=y))
                t_pg = timeit(lambda: ops.pgemm(x, w, out=y))
                err = (ops.pgemm(x, w).float() - torch.matmul(x, w.t()).float()).abs().max().item()
            r = {"shape": name, "M": M, "N": N, "K": K, "lib_us": round(t_lib * 1e6, 1),
                 "pgemm_us": round(t_pg * 1e6, 1), "hipblaslt_tflops": fl / t_lib / 1e12,
                 "pgemm_tflops": fl / t_pg / 1e12, "speedup": t_lib / t_pg, "max_err": err}
            rows.append(r)
            print(json.dumps(r), flush=True)
            del x, w, y
        DENSE.clear()
        del GROUPED[2:]
    for name, M, N, K in DENSE:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        t_lib = timeit(lambda: torch.matmul(x, w.t(), out=y))
        t_pg = timeit(lambda: ops.pgemm(x, w, out=y))
        err = (ops.pgemm(x, w).float() - torch.matmul(x, w.t()).float()).abs().max().item()
        r = {"shape": name, "M": M, "N": N, "K": K, "hipblaslt_tflops": fl / t_lib / 1e12,
             "pgemm_tflops": fl / t_pg / 1e12, "speedup": t_lib / t_pg, "max_err": err}
        rows.append(r)
        print(json.dumps(r), flush=True)
        del x, w, y
    for name, T, G, N, K in GROUPED:
        g = torch.Generator(device="cpu").manual_seed(G)
        cnt = torch.multinomial(torch.ones(G), T, replacement=True, generator=g).bincount(minlength=G)
        offs = cnt.cumsum(0).int().to(dev)
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(G, N, K, device=dev, dtype=torch.bfloat16) * 0.02
        wt = w.transpose(1, 2)
        fl = 2.0 * T * N * K
        t_lib = timeit(lambda: torch._grouped_mm(x, wt, offs=offs), iters=10)
        t_pg = timeit(lambda: ops.pgemm(x, w, offs=offs), iters=10)
        err = (ops.pgemm(x, w, offs=offs).float()
               - torch._grouped_mm(x, wt, offs=offs).float()).abs().max().item()
        r = {"shape": name, "rows": T, "experts": G, "N": N, "K": K,
             "grouped_mm_tflops": fl / t_lib / 1e12, "pgemm_tflops": fl / t_pg / 1e12,
             "speedup": t_lib / t_pg, "max_err": err}
        rows.append(r)
        print(json.dumps(r), flush=True)
        del x, w
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
