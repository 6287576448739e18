"""Decode-shape GEMM microbenchmark: hipBLASLt vs rocBLAS through torch (M = batch)."""
import sys
import torch

shapes = [(4096, 1024), (1024, 2048), (6144, 1024), (1024, 3072), (151936, 1024)]
M = int(sys.argv[1]) if len(sys.argv) > 1 else 256
for lib in ["cublaslt", "cublas"]:
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:
        print("skip", lib, e)
        continue
    tot = 0.0
    for N, K in shapes:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        for _ in range(5):
            torch.nn.functional.linear(x, w)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(50):
            torch.nn.functional.linear(x, w)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / 50
        tot += us
        print(f"{lib:9s} M={M} N={N:6d} K={K:5d}: {us:7.1f} us  {2*M*N*K/us/1e6:7.1f} TF/s  {N*K*2/us/1e6:5.2f} TB/s(w)")
    print(lib, "sum", round(tot, 1))
