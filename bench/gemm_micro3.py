"""Decode GEMM with COLD weights (as in a real decode step: every layer's weights are
read once per step and evicted by the KV stream): hand-written MFMA kernel vs hipBLASLt.

Weight copies are rotated so their total exceeds the 256 MB Infinity Cache; reports
us/GEMM and weight-stream TB/s.  python bench/gemm_micro3.py [M ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402

ops.load_native(required=True)
Ms = [int(a) for a in sys.argv[1:]] or [128, 256]
TUNABLE = os.environ.get("AKAP_TUNABLEOP", "0") == "1"
if TUNABLE:  # let TunableOp benchmark every hipBLASLt/rocBLAS solution per shape first
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_max_tuning_iterations(30)
SHAPES = {  # (N, K)
    "llama8b.qkv": (6144, 4096), "llama8b.o": (4096, 4096), "llama8b.gate_up": (28672, 4096),
    "llama8b.down": (4096, 14336), "llama8b.lm_head": (128256, 4096),
    "qwen06.qkv": (4096, 1024), "qwen06.o": (1024, 2048), "qwen06.gate_up": (6144, 1024),
    "qwen06.down": (1024, 3072),
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
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


for M in Ms:
    for name, (N, K) in SHAPES.items():
        wbytes = N * K * 2
        copies = max(2, (1 << 30) // wbytes + 1)
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        s = ops.gemm_splitk(M, N, K)
        wsp = torch.empty(max(1, s * M * N), device="cuda", dtype=torch.float32)
        iters = max(copies, 8)
        if TUNABLE:
            torch.nn.functional.linear(x, ws[0])
            torch.cuda.synchronize()
        t_bl = timed(lambda i: torch.nn.functional.linear(x, ws[i % copies]), iters)
        cnt = ops.gemm_counters(x.device)
        t_hip = timed(lambda i: torch.ops.akap.gemm(y, x, ws[i % copies], wsp, s, cnt), iters)
        t_hip2 = timed(lambda i: torch.ops.akap.gemm(y, x, ws[i % copies], wsp, s), iters)
        print(f"M={M:4d} {name:16s} N={N:6d} K={K:5d}  blaslt {t_bl:8.2f} us "
              f"({wbytes / t_bl / 1e6:5.2f} TB/s)   hip(splitk={s}) {t_hip:8.2f} us "
              f"({wbytes / t_hip / 1e6:5.2f} TB/s)  [separate reduce: {t_hip2:7.2f} us]", flush=True)
        del ws
        torch.cuda.empty_cache()
