"""A/B in one process: decode attention on a ready q (plain kernel) vs the fused kernel that
also does q/k RMSNorm + RoPE + the new token's K/V write from the raw QKV projection, plus
the standalone qk_norm_rope_cache + plain attention pair.  Interleaved rounds, median.

python bench/attn_fused_ab.py [--B 256] [--ctx 640]
"""
import argparse
import math
import os
import statistics
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
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    ops.load_native(required=True)
    dev = "cuda"
    B, D, bs, Hq, Hkv = a.B, 128, 32, a.hq, a.hkv
    G = Hq // Hkv
    torch.manual_seed(0)
    lens = torch.randint(a.ctx - 128, a.ctx + 129, (B,), dtype=torch.int32)
    nb = [math.ceil(int(x) / bs) for x in lens]
    NB = sum(nb) + 8
    bt = torch.zeros(B, 4096 // bs, dtype=torch.int32)
    i = 0
    for s, n in enumerate(nb):  # sequential blocks, as the engine's allocator hands them out
        bt[s, :n] = torch.arange(i, i + n, dtype=torch.int32)
        i += n
    kc = torch.randn(NB, Hkv, bs, D, dtype=torch.bfloat16, device=dev)
    vc = torch.randn(NB, Hkv, bs // 8, D, 8, dtype=torch.bfloat16, device=dev)
    q = torch.randn(B, Hq, D, dtype=torch.bfloat16, device=dev)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, dtype=torch.bfloat16, device=dev)
    out = torch.empty(B, Hq, D, dtype=torch.bfloat16, device=dev)
    pos = (lens - 1).to(torch.int64)
    slots = torch.tensor([int(bt[s, int(pos[s]) // bs]) * bs + int(pos[s]) % bs
                          for s in range(B)], dtype=torch.int64)
    inv = 1.0 / (1e6 ** (torch.arange(0, D, 2, dtype=torch.float32) / D))
    ang = torch.arange(4096, dtype=torch.float32)[:, None] * inv[None, :]
    cos_sin = torch.cat([ang.cos(), ang.sin()], dim=-1).to(dev)
    qw = torch.ones(D, dtype=torch.bfloat16, device=dev)
    kw = torch.ones(D, dtype=torch.bfloat16, device=dev)
    bt, lens_d, pos_d, slots_d = bt.to(dev), lens.to(dev), pos.to(dev), slots.to(dev)
    ws = ops.decode_workspace(B, Hkv, G, int(os.environ.get("AB_WS_PARTS", "1")), dev)
    scale = 1 / math.sqrt(D)
    kv_bytes = int(lens.sum()) * Hkv * D * 2 * 2
    qbuf = torch.empty(B, Hq, D, dtype=torch.bfloat16, device=dev)

    def plain():
        ops.paged_attention_decode(out, q, kc, vc, bt, lens_d, G, scale, workspace=ws,
                                   num_parts=1, part_size=4096)

    def fused():
        ops.paged_attention_decode_fused(out, qkv, kc, vc, bt, lens_d, pos_d, slots_d, cos_sin,
                                         qw, kw, G, scale, 1e-6, workspace=ws, num_parts=1,
                                         part_size=4096)

    def split():
        ops.qk_norm_rope_cache(qkv, qbuf, kc, vc, pos_d, slots_d, cos_sin, qw, kw, Hq, Hkv, 1e-6,
                               True)
        ops.paged_attention_decode(out, qbuf, kc, vc, bt, lens_d, G, scale, workspace=ws,
                                   num_parts=1, part_size=4096)

    slots_none = torch.full_like(slots_d, -1)
    vtail = torch.zeros(B, Hkv, 8, D, dtype=torch.bfloat16, device=dev)
    tslot = torch.arange(B, dtype=torch.int32, device=dev)

    def fused_nowrite():  # the prologue without the new token's K/V writes (slot -1)
        ops.paged_attention_decode_fused(out, qkv, kc, vc, bt, lens_d, pos_d, slots_none,
                                         cos_sin, qw, kw, G, scale, 1e-6, workspace=ws,
                                         num_parts=1, part_size=4096)

    def fused_tail():  # the serving form: V written through the per-sequence V tail
        ops.paged_attention_decode_fused(out, qkv, kc, vc, bt, lens_d, pos_d, slots_d, cos_sin,
                                         qw, kw, G, scale, 1e-6, workspace=ws, num_parts=1,
                                         part_size=4096, v_tail=vtail, tail_slot=tslot)

    def plain_tail():  # ready q, partial last V group read from the tail (no writes)
        ops.paged_attention_decode(out, q, kc, vc, bt, lens_d, G, scale, workspace=ws,
                                   num_parts=1, part_size=4096, v_tail=vtail, tail_slot=tslot)

    variants = {"plain attention (q ready)": plain, "plain + V tail reads": plain_tail,
                "fused prologue attention": fused, "fused, no K/V write": fused_nowrite,
                "fused + V tail (serving)": fused_tail, "qk_norm_rope_cache + plain": split}
    graphs = {}
    for k, f in variants.items():
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            f()
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(a.iters):
                f()
        graphs[k] = g
    res = {k: [] for k in variants}
    for _ in range(a.rounds):
        for k, g in graphs.items():
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1000 / a.iters)
    for k, v in res.items():
        med = statistics.median(v)
        print(f"B={B} ctx~{a.ctx} {k:30s} median {med:7.1f} us  min {min(v):7.1f} us  "
              f"{kv_bytes / med / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
