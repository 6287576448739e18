"""A/B per batch size: where the decode layer's q/k-norm + RoPE + KV write runs.

  A (before): QKV GEMM (dgemm.hip, best split-K/prefetch) -> decode attention with the fused
              prologue (paged_attn_decode_kernel FUSED)
  B (after):  qkv_rope_gemm (qkvgemm.hip, that work in the GEMM epilogue) -> plain decode
              attention on the ready q

Qwen3-0.6B shapes (16 q / 8 kv heads, d 1024), ctx ~640, interleaved rounds, median.
python bench/qkv_rope_ab.py
"""
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import reference as ref  # noqa: E402


def graph_of(f, iters):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        f()
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(iters):
            f()
    return g


def timed(gs, rounds, iters):
    res = {k: [] for k in gs}
    for _ in range(rounds):
        for k, g in gs.items():
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1000 / iters)
    return {k: statistics.median(v) for k, v in res.items()}


def main():
    ops.load_native(required=True)
    dev = "cuda"
    Hq, Hkv, D, bs, d, ctx, L = 16, 8, 128, 32, 1024, 640, 28
    G = Hq // Hkv
    iters, rounds = 10, 5
    ws_l = [torch.randn((Hq + 2 * Hkv) * D, d, device=dev, dtype=torch.bfloat16) * 0.03
            for _ in range(L)]
    cs = ref.rope_cos_sin(4096, D, 1e6).to(dev)
    qw = torch.ones(D, dtype=torch.bfloat16, device=dev)
    kw = torch.ones(D, dtype=torch.bfloat16, device=dev)
    for B in (16, 32, 64, 128, 256):
        lens = torch.randint(ctx - 128, ctx + 129, (B,), dtype=torch.int32)
        nb = [math.ceil(int(x) / bs) for x in lens]
        NB = sum(nb) + 8
        bt = torch.zeros(B, 4096 // bs, dtype=torch.int32)
        i = 0
        for s_, n in enumerate(nb):
            bt[s_, :n] = torch.arange(i, i + n, dtype=torch.int32)
            i += n
        kc = torch.randn(NB, Hkv, bs, D, dtype=torch.bfloat16, device=dev)
        vc = torch.randn(NB, Hkv, bs // 8, D, 8, dtype=torch.bfloat16, device=dev)
        pos = (lens - 1).to(torch.int64)
        slots = torch.tensor([int(bt[s_, int(pos[s_]) // bs]) * bs + int(pos[s_]) % bs
                              for s_ in range(B)], dtype=torch.int64)
        bt, lens_d, pos_d, slots_d = bt.to(dev), lens.to(dev), pos.to(dev), slots.to(dev)
        x = torch.randn(B, d, device=dev, dtype=torch.bfloat16)
        ss = torch.full((B,), float(d), device=dev)
        q = torch.empty(B, Hq, D, device=dev, dtype=torch.bfloat16)
        out = torch.empty(B, Hq, D, device=dev, dtype=torch.bfloat16)
        parts = 1 if B * Hkv >= 2048 else min(math.ceil(2048 / (B * Hkv)), 16)
        ps = math.ceil(math.ceil(4096 / parts) / 128) * 128
        parts = math.ceil(4096 / ps)
        wsp = ops.decode_workspace(B, Hkv, G, parts, dev)
        scale = 1 / math.sqrt(D)
        li = [0]

        def gemm_cfg(s, pf, bn=0):
            def f():
                w = ws_l[li[0] % L]
                li[0] += 1
                return ops.dgemm(x, w, splitk=s, pf=pf, bn=bn, eps=1e-6, ss_in=ss)
            return f

        cands = {}
        for s in (1, 2, 4, 8):
            for pf in (2, 4):
                if ops.dgemm_supported(B, (Hq + 2 * Hkv) * D, d, s, pf):
                    cands[f"s{s}p{pf}"] = gemm_cfg(s, pf)
            if ops.dgemm_supported(B, (Hq + 2 * Hkv) * D, d, s, 1, bn=64):
                cands[f"s{s}g64"] = gemm_cfg(s, 1, 64)
        tg = timed({k: graph_of(f, iters) for k, f in cands.items()}, 3, iters)
        best = min(tg, key=tg.get)
        gemm = cands[best]

        def path_a():
            qkv = gemm()
            ops.paged_attention_decode_fused(out, qkv, kc, vc, bt, lens_d, pos_d, slots_d, cs,
                                             qw, kw, G, scale, 1e-6, workspace=wsp,
                                             num_parts=parts, part_size=ps)

        def path_b(bm, ns):
            def f():
                w = ws_l[li[0] % L]
                li[0] += 1
                ops.qkv_rope_gemm(x, w, q, kc, vc, pos_d, slots_d, cs, qw, kw, Hq, Hkv, 1e-6,
                                  ss_in=ss, bm=bm, ns=ns)
                ops.paged_attention_decode(out, q, kc, vc, bt, lens_d, G, scale, workspace=wsp,
                                           num_parts=parts, part_size=ps)
            return f

        def rope_only(bm, ns):
            def f():
                w = ws_l[li[0] % L]
                li[0] += 1
                ops.qkv_rope_gemm(x, w, q, kc, vc, pos_d, slots_d, cs, qw, kw, Hq, Hkv, 1e-6,
                                  ss_in=ss, bm=bm, ns=ns)
            return f

        def path_c():
            qkv = gemm()
            ops.qk_norm_rope_cache(qkv, q, kc, vc, pos_d, slots_d, cs, qw, kw, Hq, Hkv, 1e-6,
                                   True, decode=True)
            ops.paged_attention_decode(out, q, kc, vc, bt, lens_d, G, scale, workspace=wsp,
                                       num_parts=parts, part_size=ps)

        def rope_kernel():
            ops.qk_norm_rope_cache(qkv_buf, q, kc, vc, pos_d, slots_d, cs, qw, kw, Hq, Hkv, 1e-6,
                                   True, decode=True)

        def attn_only():
            ops.paged_attention_decode(out, q, kc, vc, bt, lens_d, G, scale, workspace=wsp,
                                       num_parts=parts, part_size=ps)

        qkv_buf = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
        variants = {f"A gemm {best} + fused attn": path_a, f"gemm {best} alone": gemm,
                    f"C gemm {best} + decode rope kernel + attn": path_c,
                    "decode rope kernel alone": rope_kernel, "plain attn alone": attn_only}
        for bm, ns in ((32, 3), (32, 6), (64, 3), (64, 6)):
            variants[f"B qkv_rope bm{bm} ns{ns} + attn"] = path_b(bm, ns)
            variants[f"qkv_rope bm{bm} ns{ns} alone"] = rope_only(bm, ns)
        t = timed({k: graph_of(f, iters) for k, f in variants.items()}, rounds, iters)
        print(f"B={B} parts={parts}: " + "  ".join(f"[{k}] {v:.1f}" for k, v in t.items()),
              flush=True)


if __name__ == "__main__":
    main()
