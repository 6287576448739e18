"""Can the HBM-bound decode attention hide the latency-bound GEMM chain?

Two half-batches (micro-batches) of a Qwen3-0.6B decode step, captured in hipGraphs:
  seq     : both halves one after the other on one stream (fused GEMM chain + attention)
  full    : the whole batch in one forward (what the engine runs today)
  overlap : the halves on two HIP streams, attention kernels forced to alternate
            (attn(A, l) -> attn(B, l) -> attn(A, l+1) ...) so each half's GEMMs run while
            the other half streams its KV cache.
python bench/overlap_micro.py [--B 256] [--ctx 640]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.models.config import get_config  # noqa: E402
from aws_k8s_ansible_provisioner_amd.models.transformer import AttnBatch, DecoderLM  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner  # noqa: E402


def make_batch(m, B, ctx, dev, BS=32):
    lens = torch.randint(ctx - 128, ctx + 129, (B,), dtype=torch.int32)
    nb = [math.ceil(int(x) / BS) for x in lens]
    NB = sum(nb) + 8
    kv = m.allocate_kv_cache(NB, BS)
    kc, vc = m.cache_views(kv, BS)
    perm = torch.randperm(NB)
    bt = torch.zeros(B, 4096 // BS, dtype=torch.int32)
    i = 0
    for s, n in enumerate(nb):
        bt[s, :n] = perm[i:i + n].to(torch.int32)
        i += n
    pos = (lens - 1).to(torch.int64)
    slots = torch.tensor([int(bt[s, int(pos[s]) // BS]) * BS + int(pos[s]) % BS
                          for s in range(B)], dtype=torch.int64)
    d = lambda t: t.to(dev)  # noqa: E731
    ws = ops.decode_workspace(B, m.hkv, m.hq // m.hkv, 1, dev)
    batch = AttnBatch(False, d(pos), d(slots), d(bt), d(lens),
                      d(torch.arange(B + 1, dtype=torch.int32)), None, None, 1, 4096, ws)
    ids = torch.randint(0, m.cfg.vocab_size, (B,), device=dev)
    return batch, ids, kc, vc, kv


class Half:
    """Per-micro-batch state of the layer-split fused forward."""

    def __init__(self, m, batch, ids, kc, vc, plan):
        self.m, self.batch, self.ids, self.kc, self.vc, self.plan = m, batch, ids, kc, vc, plan

    def start(self):
        m = self.m
        T = self.ids.shape[0]
        self.T = T
        self.residual = m.embed_tokens(self.ids)
        self.ss = torch.zeros(2 * len(m.layers), T, dtype=torch.float32, device=m.device)
        self.a1 = ops.rms_norm(self.residual, m.layers[0].ln1, m.cfg.rms_eps)
        self.ss_in = None

    def pre(self, li):
        m, lw = self.m, self.m.layers[li]
        s_, p_ = self.plan["w_qkv"][:2]
        self.qkv = ops.dgemm(self.a1, lw.w_qkv, splitk=s_, pf=p_, eps=m.cfg.rms_eps,
                             ss_in=self.ss_in)

    def attn(self, li):
        m, lw, b = self.m, self.m.layers[li], self.batch
        self.at = torch.empty(self.T, m.hq, m.D, dtype=m.dtype, device=m.device)
        ops.paged_attention_decode_fused(
            self.at, self.qkv, self.kc[li], self.vc[li], b.block_tables, b.seq_lens,
            b.positions, b.slots, m.cos_sin, lw.q_norm, lw.k_norm, m.hq // m.hkv, m.scale,
            m.cfg.rms_eps, workspace=b.workspace, num_parts=b.num_parts, part_size=b.part_size)

    def post(self, li):
        m, lw, eps, T = self.m, self.m.layers[li], self.m.cfg.rms_eps, self.T
        a2 = torch.empty_like(self.residual)
        s_, p_ = self.plan["w_o"][:2]
        ops.dgemm(self.at.view(T, m.hq * m.D), lw.w_o, splitk=s_, pf=p_, eps=eps,
                  out=self.residual, epi=ops.EPI_RESNORM, ss_out=self.ss[2 * li], a_out=a2,
                  ln_out=lw.ln2)
        s_, p_ = self.plan["w_gate_up"][:2]
        act = ops.dgemm(a2, lw.w_gate_up, splitk=s_, pf=p_, eps=eps, ss_in=self.ss[2 * li],
                        epi=ops.EPI_SILU)
        s_, p_ = self.plan["w_down"][:2]
        if li + 1 < len(m.layers):
            self.a1 = torch.empty_like(self.residual)
            ops.dgemm(act, lw.w_down, splitk=s_, pf=p_, eps=eps, out=self.residual,
                      epi=ops.EPI_RESNORM, ss_out=self.ss[2 * li + 1], a_out=self.a1,
                      ln_out=m.layers[li + 1].ln1)
            self.ss_in = self.ss[2 * li + 1]
        else:
            x = ops.dgemm(act, lw.w_down, splitk=s_, pf=p_, eps=eps)
            self.h, _ = ops.fused_add_rms_norm(x, self.residual, m.final_norm, eps)


def run_seq(halves):
    for h in halves:
        h.start()
        for li in range(len(h.m.layers)):
            h.pre(li)
            h.attn(li)
            h.post(li)


_KEEP = []
SYNC = os.environ.get("OVERLAP_SYNC", "fresh")  # fresh | events | waitstream | oneway | none


def run_overlap(halves, streams):
    main = torch.cuda.current_stream()
    L = len(halves[0].m.layers)
    ev = [[torch.cuda.Event() for _ in range(L)] for _ in halves]
    _KEEP.append(ev)  # captured event nodes must outlive the capture
    for s in streams:
        s.wait_stream(main)
    for k, h in enumerate(halves):
        with torch.cuda.stream(streams[k]):
            h.start()
    for li in range(L):
        for k, h in enumerate(halves):
            with torch.cuda.stream(streams[k]):
                h.pre(li)
                # attention kernels alternate A_l, B_l, A_{l+1}: each runs alone on the HBM
                # while the other half's GEMMs fill in
                if SYNC == "events":
                    if k == 1:
                        streams[k].wait_event(ev[0][li])
                    elif li > 0:
                        streams[k].wait_event(ev[1][li - 1])
                elif SYNC == "oneway":
                    if k == 1:
                        streams[k].wait_event(ev[0][li])
                elif SYNC == "waitstream":
                    if k == 1:
                        streams[1].wait_stream(streams[0])
                    elif li > 0:
                        streams[0].wait_stream(streams[1])
                h.attn(li)
                if (SYNC == "events" and (k == 0 or li + 1 < L)) or (SYNC == "oneway" and k == 0):
                    ev[k][li].record(streams[k])
                h.post(li)
    for s in streams:
        main.wait_stream(s)


def run_fresh_range(halves, pool, l0, l1):
    """run_fresh over layers [l0, l1) (state carried in the Half objects)."""
    main = torch.cuda.current_stream()
    it = iter(pool)
    cur = [next(it) for _ in halves]
    for s in cur:
        s.wait_stream(main)
    if l0 == 0:
        for k, h in enumerate(halves):
            with torch.cuda.stream(cur[k]):
                h.start()
    last = None
    for li in range(l0, l1):
        for k, h in enumerate(halves):
            with torch.cuda.stream(cur[k]):
                h.pre(li)
            if last is not None:
                ns = next(it)
                ns.wait_stream(cur[k])
                ns.wait_event(last)
                cur[k] = ns
            with torch.cuda.stream(cur[k]):
                h.attn(li)
            last = torch.cuda.Event()
            last.record(cur[k])
            _KEEP.append(last)
            with torch.cuda.stream(cur[k]):
                h.post(li)
    for s in cur:
        main.wait_stream(s)


def timed_graphs(fns, iters=10):
    """Capture each fn in its own graph; time replaying them back to back."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for fn in fns:
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    pool = torch.cuda.graph_pool_handle()
    gs = []
    for fn in fns:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool):
            fn()
        gs.append(g)
    for g in gs:
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(iters):
        for g in gs:
            g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


def run_fresh(halves, pool):
    """Alternating attention with only forward stream dependencies: every cross-stream wait
    continues on a brand-new stream (hipGraph capture on ROCm 7 segfaults when a stream waits
    on a stream that earlier waited on it: bench/graph_multistream_probe.py)."""
    main = torch.cuda.current_stream()
    it = iter(pool)
    L = len(halves[0].m.layers)
    cur = [next(it) for _ in halves]
    for s in cur:
        s.wait_stream(main)
    for k, h in enumerate(halves):
        with torch.cuda.stream(cur[k]):
            h.start()
    last = None
    for li in range(L):
        for k, h in enumerate(halves):
            with torch.cuda.stream(cur[k]):
                h.pre(li)
            if last is not None:
                ns = next(it)
                ns.wait_stream(cur[k])
                ns.wait_event(last)
                cur[k] = ns
            with torch.cuda.stream(cur[k]):
                h.attn(li)
            last = torch.cuda.Event()
            last.record(cur[k])
            _KEEP.append(last)
            with torch.cuda.stream(cur[k]):
                h.post(li)
    for s in cur:
        main.wait_stream(s)


def run_attnstream(halves, streams, sa):
    """Attention kernels of both halves on their own stream (serialised A0 B0 A1 B1 ...);
    each half's GEMMs on its stream."""
    main = torch.cuda.current_stream()
    L = len(halves[0].m.layers)
    for s in list(streams) + [sa]:
        s.wait_stream(main)
    for k, h in enumerate(halves):
        with torch.cuda.stream(streams[k]):
            h.start()
    for li in range(L):
        for k, h in enumerate(halves):
            with torch.cuda.stream(streams[k]):
                h.pre(li)
            sa.wait_stream(streams[k])
            with torch.cuda.stream(sa):
                h.attn(li)
            streams[k].wait_stream(sa)
            with torch.cuda.stream(streams[k]):
                h.post(li)
    for s in list(streams) + [sa]:
        main.wait_stream(s)


def timed_graph(fn, iters=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-0.6b")
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--ctx", type=int, default=640)
    a = ap.parse_args()
    ops.load_native(required=True)
    dev = torch.device("cuda", 0)
    m = DecoderLM(get_config(a.model), dev, max_model_len=4096)
    H = a.B // 2
    gemm_tuner.tune_model(m, [H, a.B])
    gemm_tuner.tune_fused(m, [H, a.B])
    plan_h, plan_f = gemm_tuner.fused_plan(H), gemm_tuner.fused_plan(a.B)
    parts = [make_batch(m, H, a.ctx, dev) for _ in range(2)]
    halves = [Half(m, b, i, kc, vc, plan_h) for (b, i, kc, vc, _) in parts]
    full_b, full_ids, fkc, fvc, _ = make_batch(m, a.B, a.ctx, dev)
    print("timing full", flush=True)
    t_full = timed_graph(lambda: m._forward_fused_decode(full_ids, full_b, fkc, fvc, plan_f))
    print("timing seq", flush=True)
    t_seq = timed_graph(lambda: run_seq(halves))
    print("timing overlap", flush=True)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    if SYNC == "fresh":
        pool = [torch.cuda.Stream() for _ in range(4 * len(m.layers) + 4)]
        G = int(os.environ.get("OVERLAP_GROUP", "7"))
        L = len(m.layers)
        fns = [lambda l0=l0: run_fresh_range(halves, pool, l0, min(L, l0 + G))
               for l0 in range(0, L, G)]
        t_ov = timed_graphs(fns)
    elif SYNC == "attnstream":
        sa = torch.cuda.Stream()
        t_ov = timed_graph(lambda: run_attnstream(halves, streams, sa))
    else:
        t_ov = timed_graph(lambda: run_overlap(halves, streams))
    # same numbers either way?
    run_seq(halves)
    ref = [h.h.clone() for h in halves]
    if SYNC == "fresh":
        for fn in fns:
            fn()
    else:
        run_overlap(halves, streams)
    torch.cuda.synchronize()
    same = all(torch.equal(r, h.h) for r, h in zip(ref, halves))
    print(f"B={a.B} ctx~{a.ctx}: full {t_full:.1f} us, halves sequential {t_seq:.1f} us, "
          f"halves overlapped {t_ov:.1f} us  (overlap/full {t_ov / t_full:.3f}; "
          f"results identical: {same})", flush=True)


if __name__ == "__main__":
    main()
