"""L2 behaviour of the prefill GEMMs: hipBLASLt vs pgemm on the same shapes (run under
rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum; the per-kernel counters give the L2 hit rate and
the bytes fetched past L2).  Shapes: Qwen3-0.6B qkv (K 1024) and Llama-3-8B qkv (K 4096) at
M = 16384.
    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d OUT -o run -- \
        python3 tools/gemm_l2_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402

for M, N, K in ((16384, 4096, 1024), (16384, 6144, 4096)):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.matmul(x, w.t(), out=y)
        ops.pgemm(x, w, out=y)
    torch.cuda.synchronize()
    print(f"done {M}x{N}x{K}", flush=True)
