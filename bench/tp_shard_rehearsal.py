"""One tensor-parallel rank of Llama-3-70B TP=8 on ONE MI355X, collectives stubbed.

The 8-GPU TP run needs a whole node; this instantiates the real per-rank shard that
`bench.py --tp 8 --model llama-3-70b` builds on each GPU (8 of 64 q heads, 1 of 8 kv heads,
d 8192, 3584 of 28672 FFN columns, 16,032 of 128,256 vocab rows: 17.6 GB of bf16 weights)
and times its compute. Shapes, kernels, GEMM tuner choices and hipGraph capture are
identical. The TP collectives are replaced by local stand-ins of the same shape:
  tp_all_reduce           the custom all-reduce kernel on a one-rank communicator
  tp_all_reduce_resnorm   the same kernel with its fused residual + next-norm epilogue
  tp_all_gather_last      the custom IPC all-gather kernel on the same communicator, then the
                          shard repeated tp times
so the result is a per-rank compute time including the all-reduce launches; a TP step adds
the xGMI exchange of two B x 8192 bf16 all-reduces per layer to it.

python bench/tp_shard_rehearsal.py [--model llama-3-70b] [--tp 8] [--B 64,128,256] [--ctx 1024]
"""
import argparse
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.models.config import get_config  # noqa: E402
from aws_k8s_ansible_provisioner_amd.models.transformer import AttnBatch, DecoderLM  # noqa: E402
from aws_k8s_ansible_provisioner_amd.parallel import comm, state  # noqa: E402


def stub_collectives(tp: int) -> None:
    """Local stand-ins of the TP collectives.  The all-reduces run the REAL custom all-reduce
    kernels (csrc/kernels/custom_allreduce.hip) on a one-rank communicator: the same launch,
    staging, flag protocol and fused residual + next-norm epilogue, minus the peer reads over
    xGMI -- so the per-rank step includes the all-reduce kernels' own cost, not a chain of
    Python elementwise stand-ins (which inflated round 2's number by ~6 ms at B=256)."""
    h = torch.ops.akap.car_create(torch.cuda.current_device(), 0, 1, 1 << 23)
    torch.ops.akap.car_link_local(h, [h])

    def all_reduce(x):
        if x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() % 8 == 0:
            torch.ops.akap.car_all_reduce(h, x, x, False)
        return x

    def resnorm(partial, residual, ln, a_out, ss):
        torch.ops.akap.car_all_reduce_resnorm(h, partial, residual, ln, a_out, ss, False)

    def all_gather_last(x, out=None):
        # the real IPC all-gather kernel (one-rank communicator: the own shard's staging
        # write, flag exchange and store), then the shard repeated to the full width
        flat = x.contiguous().view(-1, x.shape[-1])
        mine = torch.empty_like(flat)
        torch.ops.akap.car_all_gather(h, flat, mine)
        return torch.cat([mine.view_as(x)] * tp, dim=-1)

    comm.tp_all_reduce = all_reduce
    comm.tp_all_reduce_resnorm = resnorm
    comm.tp_all_gather_last = all_gather_last


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-70b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--B", default="64,128,256")
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    ops.load_native(required=True)
    dev = torch.device("cuda", 0)
    cfg = get_config(a.model)
    # rank 0 of a TP group; world_size 1 so object broadcasts stay local
    ps = state.ParallelState(rank=0, world_size=1, tp_size=a.tp, tp_rank=0)
    state.set_state(ps)
    stub_collectives(a.tp)
    t0 = time.time()
    m = DecoderLM(cfg, dev, pstate=ps, max_model_len=4096)
    nparam = sum(p.numel() for p in [m.embed, m.lm_head] if p is not None) + sum(
        t.numel() for lw in m.layers for t in (lw.w_qkv, lw.w_o, lw.w_gate_up, lw.w_down))
    print(f"{a.model} TP={a.tp} rank 0 shard: hq {m.hq} hkv {m.hkv} d {cfg.hidden_size} "
          f"ffn/rank {m.layers[0].w_down.shape[1]} vocab/rank {m.lm_head.shape[0]}: "
          f"{nparam * 2 / 1e9:.1f} GB bf16 weights, built in {time.time() - t0:.1f}s", flush=True)
    from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner
    Bs = [int(x) for x in a.B.split(",")]
    gemm_tuner.tune_model(m, Bs, log=lambda *x: print(*x, flush=True))
    gemm_tuner.tune_fused(m, Bs, log=lambda *x: print(*x, flush=True))
    BS = 32
    for B in Bs:
        lens = torch.full((B,), a.ctx, dtype=torch.int32)
        nb = [math.ceil(int(x) / BS) for x in lens]
        NB = sum(nb) + 8
        kv = m.allocate_kv_cache(NB, BS)
        kc, vc = m.cache_views(kv, BS)
        bt = torch.zeros(B, 4096 // BS, dtype=torch.int32)
        i = 0
        for s, n in enumerate(nb):
            bt[s, :n] = torch.arange(i, i + n, dtype=torch.int32)
            i += n
        pos = (lens - 1).to(torch.int64)
        slots = torch.tensor([int(bt[s, int(pos[s]) // BS]) * BS + int(pos[s]) % BS
                              for s in range(B)], dtype=torch.int64)
        d = lambda t: t.to(dev)  # noqa: E731
        parts = 1 if B * m.hkv >= 2048 else min(math.ceil(2048 / (B * m.hkv)), 16)
        ps_ = math.ceil(math.ceil(4096 / parts) / 128) * 128
        parts = math.ceil(4096 / ps_)
        ws = ops.decode_workspace(B, m.hkv, m.hq // m.hkv, parts, dev)
        batch = AttnBatch(False, d(pos), d(slots), d(bt), d(lens),
                          d(torch.arange(B + 1, dtype=torch.int32)), None, None, parts, ps_, ws)
        ids = torch.randint(0, cfg.vocab_size, (B,), device=dev)
        z = torch.zeros(B, device=dev)
        zi = torch.zeros(B, dtype=torch.int32, device=dev)
        one = torch.ones(B, device=dev)
        seeds = torch.zeros(B, dtype=torch.int64, device=dev)

        def step():
            h = m.forward(ids, batch, kc, vc)
            ops.sample(m.compute_logits(h), z, zi, one, seeds, zi)

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
        ms = e0.elapsed_time(e1) / a.iters
        fused = "fused chain" if gemm_tuner.fused_plan(B) is not None else "unfused"
        print(f"B={B} ctx={a.ctx}: per-rank decode step {ms:.2f} ms ({fused}; collectives "
              f"stubbed) -> {B / ms * 1000:.0f} tok/s per TP group before communication",
              flush=True)
        del kv, kc, vc, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
