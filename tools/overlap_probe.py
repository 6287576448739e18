"""Two-batch overlap probe: can a decode step's latency-bound GEMM chain hide under the
bandwidth-bound paged attention if the batch is split in two halves on two HIP streams?

Qwen3-0.6B decode shapes at B = 256 (ctx 640: the headline bench's mean context), 28 layers,
each layer = paged attention (our kernel) + the qkv / o / gate_up / down projections
(torch.matmul here: only the overlap is measured, not the GEMM kernels).  Variants, each
captured in ONE hipGraph and replayed:
  serial    attn(256) -> chain(256) per layer, one stream
  halves    attn(A) chain(A) attn(B) chain(B) per layer, one stream (the split's own cost)
  overlap   stream 1: attn(A) attn(B) ...; stream 2: chain(A) after attn(A), chain(B) after
            attn(B); attn(A) of layer l+1 waits for chain(A) of layer l
and the same overlap variant run eagerly (no graph) to see whether graph branches run
concurrently at all.  Prints ms per step for each.
"""
from __future__ import annotations

import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=28)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--ctx", type=int, default=640)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda")
    ops.load_native(required=True)
    L, B, ctx = a.layers, a.batch, a.ctx
    hq, hkv, D, BS = 16, 8, 128, 32
    d, F = 1024, 3072
    nbs = math.ceil(ctx / BS)
    NB = B * nbs
    bt = torch.randperm(NB, device=dev).to(torch.int32).view(B, nbs)
    sl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
    kcs = [torch.randn(NB, hkv, BS, D, device=dev, dtype=torch.bfloat16) for _ in range(L)]
    vcs = [torch.randn(NB, hkv, BS // 8, D, 8, device=dev, dtype=torch.bfloat16) for _ in range(L)]
    G = hq // hkv
    scale = 1 / math.sqrt(D)

    def wts():
        s = 0.02
        return (torch.randn((hq + 2 * hkv) * D, d, device=dev, dtype=torch.bfloat16) * s,
                torch.randn(d, hq * D, device=dev, dtype=torch.bfloat16) * s,
                torch.randn(2 * F, d, device=dev, dtype=torch.bfloat16) * s,
                torch.randn(d, F, device=dev, dtype=torch.bfloat16) * s)

    W = [wts() for _ in range(L)]
    halves = {"all": (0, B), "A": (0, B // 2), "B": (B // 2, B)}
    st = {}
    for k, (lo, hi) in halves.items():
        n = hi - lo
        st[k] = dict(q=torch.randn(n, hq, D, device=dev, dtype=torch.bfloat16),
                     o=torch.empty(n, hq, D, device=dev, dtype=torch.bfloat16),
                     x=torch.randn(n, d, device=dev, dtype=torch.bfloat16),
                     ws=ops.decode_workspace(n, hkv, G, 1, dev), bt=bt[lo:hi], sl=sl[lo:hi])

    def attn(l, k):
        s = st[k]
        ops.paged_attention_decode(s["o"], s["q"], kcs[l], vcs[l], s["bt"], s["sl"], G, scale,
                                   workspace=s["ws"], num_parts=1, part_size=1024)

    def chain(l, k):
        s = st[k]
        wqkv, wo, wgu, wd = W[l]
        h = s["o"].view(-1, hq * D) @ wo.t()
        gu = (s["x"] + h) @ wgu.t()
        m = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
        y = m @ wd.t()
        qkv = (s["x"] + y) @ wqkv.t()
        s["q"].copy_(qkv[:, :hq * D].view(-1, hq, D))

    s2 = torch.cuda.Stream()
    evs = [[torch.cuda.Event() for _ in range(4)] for _ in range(L)]

    def serial():
        for l in range(L):
            attn(l, "all")
            chain(l, "all")

    def split_serial():
        for l in range(L):
            for k in ("A", "B"):
                attn(l, k)
                chain(l, k)

    def overlap():
        main = torch.cuda.current_stream()
        for l in range(L):
            e = evs[l]
            attn(l, "A")
            e[0].record(main)
            s2.wait_event(e[0])
            with torch.cuda.stream(s2):
                chain(l, "A")
                e[1].record(s2)
            if l:
                main.wait_event(evs[l - 1][3])  # attn(B, l) needs chain(B, l - 1)
            attn(l, "B")
            e[2].record(main)
            s2.wait_event(e[2])
            with torch.cuda.stream(s2):
                chain(l, "B")
                e[3].record(s2)
            main.wait_event(e[1])  # attn(A, l+1) needs chain(A, l)
        main.wait_event(evs[L - 1][3])

    def timeit(fn, graph: bool) -> float:
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        run = fn
        if graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fn()
            run = g.replay
            run()
            torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.reps):
            run()
        t1.record()
        torch.cuda.synchronize()
        return t0.elapsed_time(t1) / a.reps

    def attn_only():
        for l in range(L):
            attn(l, "all")

    def chain_only():
        for l in range(L):
            chain(l, "all")

    res = {}
    for name, fn in [("attn_only", attn_only), ("chain_only", chain_only), ("serial", serial),
                     ("halves", split_serial), ("overlap", overlap)]:
        res[name] = timeit(fn, graph=True)
        print(f"{name:12s} graph {res[name]:8.3f} ms/step", flush=True)
    print(f"{'overlap':12s} eager {timeit(overlap, graph=False):8.3f} ms/step", flush=True)
    kv = 2 * L * B * ctx * hkv * D * 2
    print(f"attention KV bytes/step {kv / 1e9:.2f} GB -> {kv / res['attn_only'] / 1e9:.2f} TB/s",
          flush=True)


if __name__ == "__main__":
    main()
