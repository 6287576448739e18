"""Plain-PyTorch (fp32-accumulating) reference implementations of every kernel.

They define the semantics the HIP kernels are tested against and serve the CPU
engine path.  Cache layouts (BS % 32 == 0, D = 128 on the GPU path):
  K [NB, Hkv, BS, D] shape, stored MFMA-fragment ordered inside each 32-token chunk:
    [BS/32][tile tt 2][k-step D/32][row r 16][32 dims], chunk token o = 8*(r>>2)+4*tt+(r&3)
    (csrc/kernels/common.h k_swz_offset) -- use k_tokens()/write_k() to index it;
  V [NB, Hkv, BS/8, D, 8] (8-token groups, dim-major).
"""
from __future__ import annotations

import math
from typing import Optional

import torch


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(dim=-1, keepdim=True) + eps)
    return (xf * inv * w.float()).to(x.dtype)


def silu_and_mul(x: torch.Tensor) -> torch.Tensor:
    F = x.shape[-1] // 2
    g, u = x[..., :F], x[..., F:]
    return (torch.nn.functional.silu(g.float()).to(x.dtype).float() * u.float()).to(x.dtype)


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, scaling: dict | None = None,
                 device=None) -> torch.Tensor:
    """fp32 table [max_pos, D] = [cos | sin] for NeoX-style (rotate-half) rotary."""
    inv_freq = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo = scaling.get("low_freq_factor", 1.0)
        hi = scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        low_wl, high_wl = old / lo, old / hi
        wl = 2 * math.pi / inv_freq
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > low_wl, inv_freq / factor, inv_freq)
        mid = (wl <= low_wl) & (wl >= high_wl)
        scaled = torch.where(mid, (1 - smooth) * inv_freq / factor + smooth * inv_freq, scaled)
        inv_freq = scaled
    t = torch.arange(max_pos, dtype=torch.float64)
    freqs = torch.outer(t, inv_freq)
    cs = torch.cat([freqs.cos(), freqs.sin()], dim=-1).float()
    return cs.to(device) if device is not None else cs


def apply_rope(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x [T, H, D] (float) -> rotated (float)."""
    D = x.shape[-1]
    half = D // 2
    cs = cos_sin[positions.long()]
    c = cs[:, None, :half]
    s = cs[:, None, half:]
    x1, x2 = x[..., :half], x[..., half:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


FP8_MAX = 448.0  # OCP e4m3fn


def to_cache(vals: torch.Tensor, cache: torch.Tensor) -> torch.Tensor:
    """Values -> the cache's storage: bf16, or OCP e4m3fn bytes (uint8 cache, scale 1,
    clamped to +-448, round-to-nearest-even like the kernels)."""
    if cache.dtype == torch.uint8:
        f8 = vals.float().clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
        return f8.view(torch.uint8)
    return vals.to(cache.dtype)


def from_cache(t: torch.Tensor) -> torch.Tensor:
    """Cache storage -> values (fp8 bytes widen exactly to bf16)."""
    if t.dtype == torch.uint8:
        return t.view(torch.float8_e4m3fn).to(torch.bfloat16)
    return t


def k_swz(o: int) -> tuple[int, int, int]:
    """Token offset within a block -> (32-token chunk, tile tt, row r) of the K layout."""
    c, oo = divmod(o, 32)
    return c, (oo >> 2) & 1, ((oo >> 3) << 2) | (oo & 3)


# position (tt * 16 + r) of chunk token o, for o = 0..31
K_CHUNK_POS = [k_swz(o)[1] * 16 + k_swz(o)[2] for o in range(32)]


def k_blocks_view(k_cache: torch.Tensor) -> torch.Tensor:
    NB, H, BS, D = k_cache.shape
    assert BS % 32 == 0 and D % 32 == 0, "K cache layout needs BS % 32 == 0"
    return k_cache.view(NB, H, BS // 32, 2, D // 32, 16, 32)


def write_k(k_cache: torch.Tensor, b: int, o: int, val: torch.Tensor) -> None:
    """k_cache[block b, :, token o, :] = val [Hkv, D] in the swizzled layout."""
    c, tt, r = k_swz(o)
    H, D = val.shape
    k_blocks_view(k_cache)[b, :, c, tt, :, r, :] = to_cache(val, k_cache).view(H, D // 32, 32)


def k_tokens(k_cache: torch.Tensor, blocks: torch.Tensor) -> torch.Tensor:
    """Logical K of `blocks` in token order: [len(blocks) * BS, Hkv, D]."""
    NB, H, BS, D = k_cache.shape
    v = k_blocks_view(k_cache)[blocks]                       # [nb, H, C, 2, D/32, 16, 32]
    nb = v.shape[0]
    t = v.permute(0, 2, 3, 5, 1, 4, 6).reshape(nb, BS // 32, 32, H, D)  # pos = tt*16 + r
    t = t[:, :, K_CHUNK_POS]
    return from_cache(t.reshape(nb * BS, H, D))


def write_cache(k: torch.Tensor, v: torch.Tensor, k_cache, v_cache, slots) -> None:
    BS = k_cache.shape[2]
    for t in range(k.shape[0]):
        s = int(slots[t])
        if s < 0:
            continue
        b, o = divmod(s, BS)
        write_k(k_cache, b, o, k[t])
        v_cache[b, :, o // 8, :, o % 8] = to_cache(v[t], v_cache)


def qk_norm_rope_cache(qkv, q_out, k_cache, v_cache, positions, slots, cos_sin, q_w, k_w, Hq,
                       Hkv, eps, apply_rope_flag=True):
    T = qkv.shape[0]
    D = k_cache.shape[3]
    q = qkv[:, : Hq * D].reshape(T, Hq, D)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].reshape(T, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].reshape(T, Hkv, D)
    if q_w is not None:
        q = rms_norm(q, q_w, eps)
    if k_w is not None:
        k = rms_norm(k, k_w, eps)
    qf, kf = q.float(), k.float()
    if apply_rope_flag:
        qf = apply_rope(qf, positions[:T], cos_sin)
        kf = apply_rope(kf, positions[:T], cos_sin)
    q_out.copy_(qf.to(q_out.dtype).reshape(q_out.shape))
    write_cache(kf.to(qkv.dtype), v, k_cache, v_cache, slots[:T])


def reshape_and_cache(k, v, k_cache, v_cache, slots):
    write_cache(k, v, k_cache, v_cache, slots)


def gather_kv(k_cache, v_cache, block_table, kv_len: int):
    """-> K [kv_len, Hkv, D], V [kv_len, Hkv, D] from the paged caches."""
    BS = k_cache.shape[2]
    nb = (kv_len + BS - 1) // BS
    blocks = block_table[:nb].long()
    K = k_tokens(k_cache, blocks)[:kv_len]
    # [nb, Hkv, BS/8, D, 8] -> [nb, BS/8, 8, Hkv, D] -> tokens
    V = v_cache[blocks].permute(0, 2, 4, 1, 3).reshape(nb * BS, v_cache.shape[1], -1)[:kv_len]
    return K, from_cache(V)


def paged_attention(q, k_cache, v_cache, block_tables, seq_lens, q_start, scale):
    """Causal attention of each sequence's new tokens over its paged context.
    q [T, Hq, D]; q_start [B+1] cumulative; seq_lens [B] (kv incl. new tokens)."""
    out = torch.zeros_like(q)
    B = seq_lens.numel()
    Hq = q.shape[1]
    Hkv = k_cache.shape[1]
    G = Hq // Hkv
    for b in range(B):
        q0, q1 = int(q_start[b]), int(q_start[b + 1])
        ql = q1 - q0
        if ql == 0:
            continue
        kv = int(seq_lens[b])
        K, V = gather_kv(k_cache, v_cache, block_tables[b], kv)
        Kf = K.float().repeat_interleave(G, dim=1)  # [kv, Hq, D]
        Vf = V.float().repeat_interleave(G, dim=1)
        qf = q[q0:q1].float()  # [ql, Hq, D]
        s = torch.einsum("qhd,khd->hqk", qf, Kf) * scale
        qpos = torch.arange(kv - ql, kv).view(-1, 1)
        kpos = torch.arange(kv).view(1, -1)
        s = s.masked_fill((kpos > qpos)[None], float("-inf"))
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("hqk,khd->qhd", p, Vf)
        out[q0:q1] = o.to(q.dtype)
    return out


def sample(logits, temperature, top_k, top_p, seeds, steps, greedy_logprobs=False):
    """Reference sampler: greedy for T<=0; else top-k, then top-p (on the top-k
    renormalised distribution), then a draw.  Draws use torch's RNG seeded per row,
    so only the distribution (not the exact token) matches the kernel."""
    B, V = logits.shape
    toks = torch.empty(B, dtype=torch.int64)
    lps = torch.empty(B, dtype=torch.float32)
    for i in range(B):
        x = logits[i].float().cpu()
        T = float(temperature[i])
        if T <= 0:
            toks[i] = int(x.argmax())
            lps[i] = float(torch.log_softmax(x, -1)[toks[i]]) if greedy_logprobs else 0.0
            continue
        z = x / T
        logp = torch.log_softmax(z, dim=-1)
        keep = torch.ones(V, dtype=torch.bool)
        k = int(top_k[i])
        if 0 < k < V:
            kth = torch.topk(z, k).values[-1]
            keep &= z >= kth
        p = float(top_p[i])
        if p < 1.0:
            zz = z.masked_fill(~keep, float("-inf"))
            probs = torch.softmax(zz, dim=-1)
            sp, si = probs.sort(descending=True)
            cum = sp.cumsum(0)
            n = int((cum < p).sum()) + 1
            thr = sp[min(n, V) - 1]
            keep &= probs >= thr
        g = torch.Generator().manual_seed(int(seeds[i]) * 1000003 + int(steps[i]))
        zz = z.masked_fill(~keep, float("-inf"))
        pr = torch.softmax(zz, dim=-1)
        t = int(torch.multinomial(pr, 1, generator=g))
        toks[i] = t
        lps[i] = float(logp[t])
    return toks.to(logits.device), lps.to(logits.device)


def embedding(ids, table, vs, ve):
    ids = ids.long()
    mask = (ids >= vs) & (ids < ve)
    local = (ids - vs).clamp(0, table.shape[0] - 1)
    out = table[local]
    return out * mask[:, None].to(out.dtype)


def moe_topk_softmax(logits, top_k, renorm=True):
    p = torch.softmax(logits.float(), dim=-1)
    w, ids = torch.topk(p, top_k, dim=-1)
    if renorm:
        w = w / w.sum(dim=-1, keepdim=True)
    return w, ids.to(torch.int32)


def moe_align(topk_ids, E, block, cap):
    flat = topk_ids.reshape(-1).long().cpu()
    n = flat.numel()
    sorted_ids = torch.full((cap,), n, dtype=torch.int32)
    offsets = torch.zeros(E + 1, dtype=torch.int32)
    acc = 0
    for e in range(E):  # ids outside [0, E) are skipped
        idx = (flat == e).nonzero().flatten()
        offsets[e] = acc
        sorted_ids[acc:acc + idx.numel()] = idx.to(torch.int32)
        acc += (idx.numel() + block - 1) // block * block
    offsets[E] = acc
    return sorted_ids.to(topk_ids.device), offsets.to(topk_ids.device), acc


def fused_moe(h, w13, w2, topk_w, topk_ids):
    """fp32 reference of the fused expert FFN (bf16 rounding at the same points as the
    kernels: after each GEMM and after silu_and_mul).  Expert ids outside [0, E) -- the
    padding rows of the expert-parallel dispatch -- contribute nothing (as in moe_align)."""
    T, d = h.shape
    E = w13.shape[0]
    out = torch.zeros(T, d, dtype=torch.float32, device=h.device)
    ids = topk_ids.long()
    for e in range(E):
        t_idx, k_idx = (ids == e).nonzero(as_tuple=True)
        if t_idx.numel() == 0:
            continue
        y1 = (h[t_idx].float() @ w13[e].float().t()).to(h.dtype)
        a = silu_and_mul(y1)
        y2 = (a.float() @ w2[e].float().t()).to(h.dtype)
        out.index_add_(0, t_idx, topk_w[t_idx, k_idx].float()[:, None] * y2.float())
    return out.to(h.dtype)


def apply_penalties(logits, rows, toks, counts, presence, frequency, repetition):
    out = logits.clone()
    for r, t, c in zip(rows.tolist(), toks.tolist(), counts.tolist()):
        x = float(out[r, t])
        rep = float(repetition[r])
        if rep != 1.0:
            x = x / rep if x > 0 else x * rep
        x -= float(frequency[r]) * c + (float(presence[r]) if c > 0 else 0.0)
        out[r, t] = x
    return out


def pgemm(x: torch.Tensor, w: torch.Tensor, silu: bool = False,
          offs: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 reference of ops.pgemm: x @ w.T (bf16-rounded), or silu(gate) * up over the
    [gate; up] halves of w; offs (cumulative row ends): rows of group g use w[g]."""
    xf = x.float()
    if offs is None:
        y = (xf @ w.float().t()).to(x.dtype)
    else:
        y = torch.empty(x.shape[0], w.shape[-2], dtype=x.dtype, device=x.device)
        lo = 0
        for g, hi in enumerate(offs.tolist()):
            if hi > lo:
                y[lo:hi] = (xf[lo:hi] @ w[g].float().t()).to(x.dtype)
            lo = hi
    return silu_and_mul(y) if silu else y
