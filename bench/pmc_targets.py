"""Short, deterministic GPU workloads for rocprofv3 hardware-counter passes (--pmc): each mode
runs one production kernel family a fixed number of times on realistic shapes, so a PMC pass
per counter group takes seconds.

  decode   Qwen3-0.6B decode step at B=256, ctx~640: paged_attn_decode_kernel (fused q/k-norm
           + RoPE + KV write), the fused dgemm/gdgemm chain, the LM head, the sampler
  prefill  Qwen3-0.6B prefill of 4 x 4096 causal tokens: paged_attn_prefill_fa_kernel + the
           prefill GEMMs
  moe      one Mixtral-8x7B MoE block (8 experts, top-2, d 4096, ffn 14336) at T=128 decode
           tokens: moe_dgemm (grouped expert GEMM, SwiGLU epilogue) + combine

python bench/pmc_targets.py --mode decode|prefill|moe [--iters N]
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

BS = 32


def _paged(B, lens, m, max_len):
    nb = [math.ceil(int(x) / BS) for x in lens]
    NB = sum(nb) + 8
    kv = m.allocate_kv_cache(NB, BS)
    kv.normal_(0, 0.5)
    kc, vc = m.cache_views(kv, BS)
    perm = torch.randperm(NB)
    bt = torch.zeros(B, max_len // BS, dtype=torch.int32)
    i = 0
    for s, n in enumerate(nb):
        bt[s, :n] = perm[i:i + n].to(torch.int32)
        i += n
    return kc, vc, bt


def decode(iters):
    from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner

    dev = torch.device("cuda", 0)
    cfg = get_config("qwen3-0.6b")
    m = DecoderLM(cfg, dev, max_model_len=4096)
    B = 256
    # the tuner's M=256 choices (profiles/r2_gemm_variants.log), fixed so the profiled run
    # holds only the decode step's own dispatches: (split-K, prefetch, LDS-DMA tile width)
    # (split-K, prefetch, LDS-DMA tile width, ring, in-launch, kgemm rows); the LM head on the
    # wide-row kernel (wgemm.hip) as the tuner picks it at M=256 (profiles/r2_bench_*.log)
    gemm_tuner._FUSED[B] = {"w_qkv": (1, 4, 0), "w_o": (1, 1, 0, 0, False, 32),
                            "w_gate_up": (1, 1, 128, 8), "w_down": (1, 1, 0, 0, False, 32)}
    gemm_tuner._PLAN[(B, m.lm_head.shape[0], m.lm_head.shape[1])] = ("wgemm",)
    lens = torch.full((B,), 640, dtype=torch.int32)
    kc, vc, bt = _paged(B, lens, m, 4096)
    pos = (lens - 1).to(torch.int64)
    slots = torch.tensor([int(bt[s, int(pos[s]) // BS]) * BS + int(pos[s]) % BS
                          for s in range(B)], dtype=torch.int64)
    d = lambda t: t.to(dev)  # noqa: E731
    ws = ops.decode_workspace(B, m.hkv, m.hq // m.hkv, 1, dev)
    batch = AttnBatch(False, d(pos), d(slots), d(bt), d(lens),
                      d(torch.arange(B + 1, dtype=torch.int32)), None, None, 1, 4096, ws)
    ids = torch.randint(0, cfg.vocab_size, (B,), device=dev)
    z = torch.zeros(B, device=dev)
    zi = torch.zeros(B, dtype=torch.int32, device=dev)

    def step():
        h = m.forward(ids, batch, kc, vc)
        ops.sample(m.compute_logits(h), z, zi, torch.ones(B, device=dev),
                   torch.zeros(B, dtype=torch.int64, device=dev), zi)

    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        step()
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        step()
    for _ in range(iters):
        g.replay()
    torch.cuda.synchronize()


def prefill(iters):
    dev = torch.device("cuda", 0)
    cfg = get_config("qwen3-0.6b")
    m = DecoderLM(cfg, dev, max_model_len=8192)
    B, P = 4, 4096
    lens = torch.full((B,), P, dtype=torch.int32)
    kc, vc, bt = _paged(B, lens, m, 8192)
    pos = torch.arange(P, dtype=torch.int64).repeat(B)
    slots = torch.cat([bt[s, torch.arange(P) // BS].to(torch.int64) * BS + torch.arange(P) % BS
                       for s in range(B)])
    q_start = torch.arange(0, B * P + 1, P, dtype=torch.int32)
    G = m.hq // m.hkv
    ts, tr = [], []
    for s in range(B):
        for r in range(0, P * G, 128):
            ts.append(s)
            tr.append(r)
    d = lambda t: t.to(dev)  # noqa: E731
    batch = AttnBatch(True, d(pos), d(slots), d(bt), d(lens), d(q_start),
                      d(torch.tensor(ts, dtype=torch.int32)), d(torch.tensor(tr, dtype=torch.int32)),
                      tile_rows=128)
    ids = torch.randint(0, cfg.vocab_size, (B * P,), device=dev)
    for _ in range(iters):
        m.forward(ids, batch, kc, vc)
    torch.cuda.synchronize()


def moe(iters):
    dev = torch.device("cuda", 0)
    E, d, F, T, K = 8, 4096, 14336, 128, 2
    w13 = (torch.randn(E, 2 * F, d, device=dev) * 0.02).to(torch.bfloat16)
    w2 = (torch.randn(E, d, F, device=dev) * 0.02).to(torch.bfloat16)
    h = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    logits = torch.randn(T, E, device=dev, dtype=torch.bfloat16)
    w, ids = ops.moe_topk_softmax(logits, K)
    for _ in range(iters):
        ops.fused_moe(h, w13, w2, w, ids)
    torch.cuda.synchronize()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="decode", choices=["decode", "prefill", "moe"])
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    ops.load_native(required=True)
    torch.manual_seed(0)
    {"decode": decode, "prefill": prefill, "moe": moe}[a.mode](a.iters)
    print(f"pmc target {a.mode} done", flush=True)
