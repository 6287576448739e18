"""LM-head GEMM at decode batch sizes on Qwen3's tied 151,936 x 1,024 table: hipBLASLt,
the wide-row weight-streaming kernel (wgemm), the 256-row LDS-DMA decode tiles (gdgemm
g128x256), and the 256 x 256 pgemm body on the table padded to a multiple of 256 rows
(152,064).  Cold weights: three copies rotate so every call streams its table from HBM.

    python tools/lmhead_probe.py
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner as gt  # noqa: E402


def main():
    ops.load_native(required=True)
    dev = "cuda"
    V, K, VP = 151936, 1024, 152064
    ws = [torch.randn(VP, K, device=dev).to(torch.bfloat16) * 0.02 for _ in range(3)]
    wv = [w[:V] for w in ws]
    floor = V * K * 2 / 6.0e6
    for M in (64, 128, 192, 256):
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        y = torch.empty(M, V, device=dev, dtype=torch.bfloat16)
        yp = torch.empty(M, VP, device=dev, dtype=torch.bfloat16)
        res = {}
        res["hipblaslt"] = gt._timed(lambda i: torch.nn.functional.linear(x, wv[i % 3]), 3)
        res["wgemm"] = gt._timed(lambda i: torch.ops.akap.wgemm(y, x, wv[i % 3]), 3)
        if ops.dgemm_supported(M, V, K, 1, 1, bn=128, bm=256):
            res["g128x256"] = gt._timed(
                gt._gd_call(M, V, K, 1, 128, 3, False, y, x, wv, 0, None, None, None, None, 256), 3)
        res["pgemm(VP)"] = gt._timed(lambda i: torch.ops.akap.pgemm(yp, x, ws[i % 3], 0, None), 3)
        tok = torch.empty(M, dtype=torch.int64, device=dev)

        def _wa(i):
            torch.ops.akap.wgemm(y, x, wv[i % 3])
            ops.argmax(y, tok)
        res["wgemm+argmax"] = gt._timed(_wa, 3)
        ref = torch.nn.functional.linear(x, wv[0]).float()
        torch.ops.akap.pgemm(yp, x, ws[0], 0, None)
        err = (yp[:, :V].float() - ref).abs().max().item()
        print(f"M={M:4d} (weight floor {floor:5.1f} us): " +
              " | ".join(f"{k} {v:6.1f}" for k, v in res.items()) + f"  pgemm max err {err:.3g}",
              flush=True)


if __name__ == "__main__":
    main()
