"""Cold-weight sweep of the custom decode GEMM's split-K factor (separate reduce pass)
against hipBLASLt.  python bench/gemm_splitk_sweep.py [M]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402

ops.load_native(required=True)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 128
SHAPES = {"llama8b.qkv": (6144, 4096), "llama8b.o": (4096, 4096),
          "llama8b.gate_up": (28672, 4096), "llama8b.down": (4096, 14336),
          "qwen06.qkv": (4096, 1024), "qwen06.o": (1024, 2048), "qwen06.down": (1024, 3072)}


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
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


for name, (N, K) in SHAPES.items():
    wbytes = N * K * 2
    copies = max(2, (1 << 30) // wbytes + 1)
    ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    iters = max(copies, 8)
    res = [f"blaslt {timed(lambda i: torch.nn.functional.linear(x, ws[i % copies]), iters):6.1f}"]
    for s in (1, 2, 4, 8, 16, 32):
        if K // s < 128:
            break
        wsp = torch.empty(max(1, s * M * N), device="cuda", dtype=torch.float32)
        t = timed(lambda i: torch.ops.akap.gemm(y, x, ws[i % copies], wsp, s), iters)
        res.append(f"s{s} {t:6.1f}")
    print(f"M={M} {name:16s} N={N:6d} K={K:5d}: " + "  ".join(res), flush=True)
    del ws
    torch.cuda.empty_cache()
