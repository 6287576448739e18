"""Custom decode GEMM vs hipBLASLt per shape (run under rocprofv3 for kernel times)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402

ops.load_native(required=True)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 256
shapes = [(4096, 1024), (1024, 2048), (6144, 1024), (1024, 3072), (151936, 1024)]
for N, K in shapes:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for name, f in [("hip", lambda: ops.linear(x, w)),
                    ("blaslt", lambda: torch.nn.functional.linear(x, w))]:
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                f()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / 100
        print(f"{name:7s} M={M} N={N:6d} K={K:5d} splitk={ops.gemm_splitk(M, N, K)}: {us:7.2f} us/gemm (graph)")
