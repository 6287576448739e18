"""Prefill attention (csrc/kernels/attention.hip paged_attn_prefill_fa_kernel) on full prefill
chunks: us per call (captured graph), causal TFLOP/s, for the 128-row (4 waves) and 256-row
(8 waves) tiles.

    python tools/attn_prefill_probe.py [--only qwen3-0.6b:32x512] [--rows 256]
"""
from __future__ import annotations

import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner as gt  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import reference as ref  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None, help="one shape, e.g. qwen3-0.6b:32x512")
    ap.add_argument("--rows", type=int, default=None, help="one tile size (128 or 256)")
    ap.add_argument("--qprep", action="store_true",
                    help="also time the kernel that norms + rotates its own q rows from QKV")
    a = ap.parse_args()
    ops.load_native(required=True)
    dev = "cuda"
    D, BS = 128, 32
    for name, hq, hkv, nseq, L in (("qwen3-0.6b", 16, 8, 32, 512), ("qwen3-0.6b", 16, 8, 4, 4096),
                                   ("llama-3-8b", 32, 8, 32, 512), ("llama-3-8b", 32, 8, 4, 4096)):
        if a.only and a.only != f"{name}:{nseq}x{L}":
            continue
        G = hq // hkv
        per = (L + BS - 1) // BS
        NB = nseq * per + 4
        kc = (torch.randn(NB, hkv, BS, D, device=dev) * 0.5).to(torch.bfloat16)
        vc = torch.randn(NB, hkv, BS // 8, D, 8, device=dev).to(torch.bfloat16)
        bt = torch.randperm(NB, device=dev)[:nseq * per].view(nseq, per).to(torch.int32)
        sl = torch.full((nseq,), L, dtype=torch.int32, device=dev)
        qs = (torch.arange(nseq + 1, device=dev) * L).to(torch.int32)
        T = nseq * L
        q = (torch.randn(T, hq, D, device=dev) * 0.5).to(torch.bfloat16)
        out = torch.empty_like(q)
        qkv = (torch.randn(T, (hq + 2 * hkv) * D, device=dev) * 0.5).to(torch.bfloat16)
        pos = torch.cat([torch.arange(L) for _ in range(nseq)]).to(torch.int64).to(dev)
        cs = ref.rope_cos_sin(L + 16, D, 1e6, device=dev)
        qw = torch.ones(D, device=dev, dtype=torch.bfloat16)
        flop = nseq * hq * (L * (L + 1) / 2) * D * 2 * 2
        res = []
        for rows in ((a.rows,) if a.rows else (128, 256)):
            ts, tr = [], []
            for s in range(nseq):
                for r in range(0, L * G, rows):
                    ts.append(s)
                    tr.append(r)
            if not os.environ.get("PROBE_UNSORTED"):  # the serving scheduler's order
                order = sorted(range(len(ts)), key=lambda i: min(L, -(-(tr[i] + rows) // G)))
                ts, tr = [ts[i] for i in order], [tr[i] for i in order]
            ts = torch.tensor(ts, dtype=torch.int32, device=dev)
            tr = torch.tensor(tr, dtype=torch.int32, device=dev)
            us = gt._timed(lambda i: ops.paged_attention_prefill(
                out, q, kc, vc, bt, sl, qs, ts, tr, G, 1 / math.sqrt(D), tile_rows=rows), 4)
            res.append(f"{rows} rows {us:7.1f} us ({flop / us / 1e6:5.0f} TF)")
            if a.qprep:
                us = gt._timed(lambda i: ops.paged_attention_prefill(
                    out, q, kc, vc, bt, sl, qs, ts, tr, G, 1 / math.sqrt(D), tile_rows=rows,
                    qprep=(qkv, pos, cs, qw, 1e-6)), 4)
                res.append(f"qprep {us:7.1f} us")
        print(f"{name} {nseq} x {L}: " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
