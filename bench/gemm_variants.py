"""Every decode-GEMM variant on the model's real, cold per-layer weights (the tuner's harness:
one captured hipGraph rotating through all layers), printed per shape, so the tuner's choice
can be read against the whole candidate field.

python bench/gemm_variants.py [--model qwen3-0.6b] [--m 64,256] [--proj w_qkv,w_o]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.models.config import get_config  # noqa: E402
from aws_k8s_ansible_provisioner_amd.models.transformer import DecoderLM  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner as gt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="qwen3-0.6b")
ap.add_argument("--m", default="64,256")
ap.add_argument("--proj", default="w_qkv,w_o,w_gate_up,w_down")
a = ap.parse_args()
ops.load_native(required=True)
m = DecoderLM(get_config(a.model), device="cuda")
L = len(m.layers)
for M in [int(v) for v in a.m.split(",")]:
    for name in a.proj.split(","):
        ws = [getattr(lw, name) for lw in m.layers]
        N, K = ws[0].shape
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16) * 0.1
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        gb = N * K * 2 / 1e9
        rows = [("hipblaslt", gt._timed(lambda i: torch.nn.functional.linear(x, ws[i % L]), L)),
                ("wgemm", gt._timed(lambda i: torch.ops.akap.wgemm(y, x, ws[i % L]), L))]
        # floor: the same launch with K cut to one 64-deep step (boundary + one round trip)
        w64 = [w[:, :64].contiguous() for w in ws]
        x64 = x[:, :64].contiguous()
        rows.append(("floor(K=64,g64)", gt._timed(
            gt._gd_call(M, N, 64, 1, 64, 0, False, y, x64, w64, 0, None, None, None, None), L)))
        for s in (1, 2, 4, 8):
            if K % (64 * s):
                continue
            for pf in (2, 4, 8):
                if ops.dgemm_supported(M, N, K, s, pf):
                    wsp = torch.empty(max(1, s * M * N), device="cuda", dtype=torch.float32)
                    rows.append((f"s{s} reg p{pf}", gt._timed(
                        lambda i, s=s, pf=pf, wsp=wsp: torch.ops.akap.dgemm(
                            y, x, ws[i % L], wsp, 0, s, pf), L)))
            for bn, ns, inl, bm in gt._gd_variants(s, (64, 128)):
                if ops.dgemm_supported(M, N, K, s, 1, bn=bn, inlaunch=inl, bm=bm):
                    rows.append((f"s{s} {gt._gd_name((bn, ns, inl, 0, bm))}", gt._timed(
                        gt._gd_call(M, N, K, s, bn, ns, inl, y, x, ws, 0, None, None, None,
                                    None, bm), L)))
            if s == 1:
                for km in (16, 32):
                    if ops.kgemm_supported(M, N, K, km):
                        rows.append((f"k{km}", gt._timed(
                            lambda i, km=km: torch.ops.akap.kgemm(y, x, ws[i % L], km, 0, 1e-6,
                                                                  None, None, None, None), L)))
        rows.sort(key=lambda r: r[1])
        print(f"M={M:4d} {name:10s} N={N:6d} K={K:6d}: " + "  ".join(
            f"{n} {t:.1f}" for n, t in rows), flush=True)
        print(f"    best {rows[0][0]} {rows[0][1]:.1f} us = {gb / rows[0][1] * 1e6 / 1e3:.2f} TB/s "
              f"weights", flush=True)
