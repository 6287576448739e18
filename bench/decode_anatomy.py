"""Decode-step anatomy: the marginal cost of each op class inside a real decode step.

Builds the model (random init), a B-sequence decode batch at ~ctx tokens of context, and
times the captured hipGraph of one decode step (forward + LM head + sampler) with op
classes knocked out one at a time (replaced by no-ops of the same output shape).  The
difference to the full step is what that op class really costs in context (cold weights,
L2 state after the attention stream, clocks), which isolated micro-benchmarks miss.

python bench/decode_anatomy.py [--model qwen3-0.6b] [--B 256] [--ctx 640]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-0.6b")
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--ctx", type=int, default=640)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--fp8", action="store_true", help="e4m3 KV cache")
    ap.add_argument("--prefill", type=int, default=0,
                    help="instead: a prefill step of B sequences x this many new tokens")
    ap.add_argument("--tp", type=int, default=1,
                    help="one TP rank's shard, collectives stubbed (bench/tp_shard_rehearsal.py)")
    a = ap.parse_args()
    ops.load_native(required=True)
    dev = torch.device("cuda", 0)
    cfg = get_config(a.model)
    pstate = None
    if a.tp > 1:
        from aws_k8s_ansible_provisioner_amd.parallel import state
        from tp_shard_rehearsal import stub_collectives
        pstate = state.ParallelState(rank=0, world_size=1, tp_size=a.tp, tp_rank=0)
        state.set_state(pstate)
        stub_collectives(a.tp)
    m = DecoderLM(cfg, dev, max_model_len=4096, pstate=pstate)
    B, BS = a.B, 32
    lens = torch.randint(a.ctx - 128, a.ctx + 129, (B,), dtype=torch.int32)
    nb = [math.ceil(int(x) / BS) for x in lens]
    NB = sum(nb) + 8
    kvd = "fp8" if a.fp8 else "auto"
    kv = m.allocate_kv_cache(NB, BS, kvd)
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
    parts = 1 if B * m.hkv >= 2048 else min(math.ceil(2048 / (B * m.hkv)), 16)
    psz = math.ceil(math.ceil(4096 / parts) / 128) * 128
    parts = math.ceil(4096 / psz)
    ws = ops.decode_workspace(B, m.hkv, m.hq // m.hkv, parts, dev)
    batch = AttnBatch(False, d(pos), d(slots), d(bt), d(lens), d(torch.arange(B + 1,
                      dtype=torch.int32)), None, None, parts, psz, ws)
    if a.prefill:
        P = a.prefill
        lens = torch.full((B,), P, dtype=torch.int32)
        NB2 = B * math.ceil(P / BS) + 8
        kv = m.allocate_kv_cache(NB2, BS, kvd)
        kc, vc = m.cache_views(kv, BS)
        bt = torch.zeros(B, 4096 // BS, dtype=torch.int32)
        perm = torch.randperm(NB2)
        nbp = math.ceil(P / BS)
        for s_ in range(B):
            bt[s_, :nbp] = perm[s_ * nbp:(s_ + 1) * nbp].to(torch.int32)
        pos = torch.arange(P, dtype=torch.int64).repeat(B)
        slots = torch.cat([bt[s_, torch.arange(P) // BS].to(torch.int64) * BS + torch.arange(P) % BS
                           for s_ in range(B)])
        q_start = torch.arange(0, B * P + 1, P, dtype=torch.int32)
        G = m.hq // m.hkv
        TR = 128 if os.environ.get("AKAP_PREFILL_FA", "1") != "0" else 64
        ts, tr = [], []
        for s_ in range(B):
            for r in range(0, P * G, TR):
                ts.append(s_)
                tr.append(r)
        batch = AttnBatch(True, d(pos), d(slots), d(bt), d(lens), d(q_start),
                          d(torch.tensor(ts, dtype=torch.int32)),
                          d(torch.tensor(tr, dtype=torch.int32)), tile_rows=TR)
        lidx = d(q_start[1:].to(torch.int64) - 1)
    ids = torch.randint(0, cfg.vocab_size, (B * (a.prefill or 1),), device=dev)
    temp = torch.zeros(B, device=dev)
    topk = torch.zeros(B, dtype=torch.int32, device=dev)
    topp = torch.ones(B, device=dev)
    seeds = torch.zeros(B, dtype=torch.int64, device=dev)
    steps = torch.zeros(B, dtype=torch.int32, device=dev)

    def step():
        h = m.forward(ids, batch, kc, vc)
        if a.prefill:
            h = h.index_select(0, lidx)
        logits = m.compute_logits(h)
        ops.sample(logits, temp, topk, topp, seeds, steps)

    orig = {k: getattr(ops, k) for k in ("paged_attention_decode", "paged_attention_decode_fused",
                                          "paged_attention_prefill",
                                          "qk_norm_rope_cache",
                                          "rms_norm", "fused_add_rms_norm", "silu_and_mul",
                                          "linear", "sample", "fused_moe")}
    noop = {
        "attention (fused: +qk-norm/rope/kv-write)": {
            "paged_attention_decode": lambda out, *a_, **k: out,
            "paged_attention_decode_fused": lambda out, *a_, **k: out,
            "paged_attention_prefill": lambda out, *a_, **k: out},
        "qk_norm_rope_cache": {"qk_norm_rope_cache": lambda qkv, q_out, *a_, **k: q_out},
        "norms": {"rms_norm": lambda x, w, eps, out=None: x,
                  "fused_add_rms_norm": lambda x, r, w, eps, out=None: (x, r)},
        "silu_and_mul": {"silu_and_mul": lambda x, out=None: x[..., : x.shape[-1] // 2]},
        "gemms (incl. LM head)": {"linear": lambda x, w, out=None: x.new_empty(x.shape[0],
                                                                               w.shape[0])},
        "sampler": {"sample": lambda logits, *a_, **k: (None, None)},
        "fused MoE experts": {"fused_moe": lambda h, *a_, **k: h},
    }

    def run(name, patch):
        for k, f in patch.items():
            setattr(ops, k, f)
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                step()
            s.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                step()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            for _ in range(a.iters):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / a.iters
        finally:
            for k, f in orig.items():
                setattr(ops, k, f)

    full = run("full", {})
    what = f"prefill {B}x{a.prefill}" if a.prefill else f"decode B={B} ctx~{a.ctx}"
    print(f"{a.model} {what}: full step {full * 1000:8.1f} us")
    for name, patch in noop.items():
        t = run(name, patch)
        print(f"  without {name:40s} {t * 1000:8.1f} us   -> costs {(full - t) * 1000:7.1f} us "
              f"({100 * (full - t) / full:4.1f} %)")


if __name__ == "__main__":
    main()
