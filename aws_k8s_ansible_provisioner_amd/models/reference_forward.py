"""Dense, cache-free fp32 reference forward (oracle for engine correctness tests).

Recomputes the whole sequence every call with plain PyTorch math on the SAME weights
as a DecoderLM instance (tp=1), independently of the paged cache, the scheduler and
the HIP kernels.
"""
from __future__ import annotations

import torch

from ..ops import reference as ref


@torch.no_grad()
def dense_logits(model, ids: list[int]) -> torch.Tensor:
    cfg = model.cfg
    dev = model.embed.device
    T = len(ids)
    t = torch.tensor(ids, dtype=torch.int64, device=dev)
    x = model.embed[t].float()
    pos = torch.arange(T, device=dev)
    D, hq, hkv = model.D, model.hq, model.hkv
    G = hq // hkv
    cs = model.cos_sin
    if T > cs.shape[0]:
        raise ValueError(f"{T} tokens exceed the model's rotary table ({cs.shape[0]} positions)")
    mask = torch.triu(torch.ones(T, T, dtype=torch.bool, device=dev), 1)

    def norm(v, w):
        return ref.rms_norm(v.to(torch.bfloat16), w, cfg.rms_eps).float()

    for lw in model.layers:
        h = norm(x, lw.ln1)
        qkv = h @ lw.w_qkv.float().t()
        q = qkv[:, : hq * D].view(T, hq, D)
        k = qkv[:, hq * D:(hq + hkv) * D].view(T, hkv, D)
        v = qkv[:, (hq + hkv) * D:].view(T, hkv, D)
        if lw.q_norm is not None:
            q = norm(q, lw.q_norm)
            k = norm(k, lw.k_norm)
        q = ref.apply_rope(q, pos, cs)
        k = ref.apply_rope(k, pos, cs)
        k = k.repeat_interleave(G, 1)
        v = v.repeat_interleave(G, 1)
        s = torch.einsum("qhd,khd->hqk", q, k) / (D ** 0.5)
        s = s.masked_fill(mask[None], float("-inf"))
        o = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), v).reshape(T, hq * D)
        x = x + o @ lw.w_o.float().t()
        h = norm(x, lw.ln2)
        if lw.moe is not None:
            moe = lw.moe
            p = torch.softmax(h @ moe.router.float().t(), -1)
            w, e = torch.topk(p, moe.K, -1)
            if moe.cfg.moe_renormalize:
                w = w / w.sum(-1, keepdim=True)
            y = torch.zeros_like(h)
            for j in range(moe.K):
                for ex in range(moe.E):
                    sel = e[:, j] == ex
                    if sel.any():
                        gu = h[sel] @ moe.w13[ex].float().t()
                        F_ = gu.shape[-1] // 2
                        a = torch.nn.functional.silu(gu[:, :F_]) * gu[:, F_:]
                        y[sel] += w[sel, j:j + 1] * (a @ moe.w2[ex].float().t())
            x = x + y
        else:
            gu = h @ lw.w_gate_up.float().t()
            F_ = gu.shape[-1] // 2
            a = torch.nn.functional.silu(gu[:, :F_]) * gu[:, F_:]
            x = x + a @ lw.w_down.float().t()
    h = norm(x, model.final_norm)
    return (h @ model.lm_head.float().t())[:, : cfg.vocab_size]


def greedy_generate(model, prompt: list[int], n: int) -> list[int]:
    ids = list(prompt)
    out = []
    for _ in range(n):
        nxt = int(dense_logits(model, ids)[-1].argmax())
        out.append(nxt)
        ids.append(nxt)
    return out
