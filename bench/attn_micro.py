"""Decode / prefill attention microbenchmark (HBM bandwidth achieved).

python bench/attn_micro.py [--B 256] [--ctx 640] [--hq 16 --hkv 8]
AKAP_ATTN_FLAGS selects kernel variants (read once per process)."""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--ctx", type=int, default=640)
    ap.add_argument("--hq", type=int, default=16)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--bs", type=int, default=32)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--spread", type=int, default=128)
    ap.add_argument("--parts", default="1,2,4,8,16")
    ap.add_argument("--fp8", action="store_true", help="e4m3 KV cache")
    a = ap.parse_args()
    ops.load_native(required=True)
    dev = "cuda"
    B, D, bs = a.B, 128, a.bs
    lens = torch.randint(a.ctx - a.spread, a.ctx + a.spread + 1, (B,), dtype=torch.int32)
    nb = [math.ceil(int(x) / bs) for x in lens]
    NB = sum(nb) + 8
    perm = torch.randperm(NB)
    mb = max(nb)
    bt = torch.zeros(B, 4096 // bs, dtype=torch.int32)
    i = 0
    for s, n in enumerate(nb):
        bt[s, :n] = perm[i:i + n].to(torch.int32)
        i += n
    kc = torch.randn(NB, a.hkv, bs, D, dtype=torch.bfloat16, device=dev)
    vc = torch.randn(NB, a.hkv, bs // 8, D, 8, dtype=torch.bfloat16, device=dev)
    if a.fp8:
        kc = kc.to(torch.float8_e4m3fn).view(torch.uint8)
        vc = vc.to(torch.float8_e4m3fn).view(torch.uint8)
    q = torch.randn(B, a.hq, D, dtype=torch.bfloat16, device=dev)
    out = torch.empty_like(q)
    bt, lens_d = bt.to(dev), lens.to(dev)
    G = a.hq // a.hkv
    kv_bytes = int(lens.sum()) * a.hkv * D * 2 * (1 if a.fp8 else 2)
    flags = os.environ.get("AKAP_ATTN_FLAGS", "default")
    for parts in [int(x) for x in a.parts.split(",")]:
        ps = 4096 // parts
        ws = ops.decode_workspace(B, a.hkv, G, parts, dev)
        f = lambda: ops.paged_attention_decode(out, q, kc, vc, bt, lens_d, G, 1 / math.sqrt(D),  # noqa
                                               workspace=ws, num_parts=parts, part_size=ps)
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / a.iters
        print(f"flags={flags} B={B} ctx~{a.ctx} parts={parts:2d} part={ps:4d}: {us:8.1f} us "
              f"{kv_bytes / us / 1e6:7.2f} TB/s")


if __name__ == "__main__":
    main()
