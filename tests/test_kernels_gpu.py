"""Numerics of the hand-written gfx950 HIP kernels vs the fp32 PyTorch references.

Every test here runs the HIP kernel (torch.ops.akap.*) on the GPU and compares it
with ops.reference on the same inputs.  Requires an MI355X.
"""
import math

import pytest
import torch

from aws_k8s_ansible_provisioner_amd import ops
from aws_k8s_ansible_provisioner_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _native():
    ops.load_native(required=True)


def _close(a, b, atol, rtol=0.0):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    lim = atol + rtol * b.abs()
    assert bool((err <= lim).all()), f"max err {err.max().item():.4g} (atol {atol})"


@pytest.mark.parametrize("d", [128, 1024, 2048, 4096, 6144, 8192, 1000])
@pytest.mark.parametrize("rows", [1, 7, 300, 1025])
def test_rmsnorm(d, rows):
    torch.manual_seed(0)
    x = torch.randn(rows, d, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(d, device=DEV, dtype=torch.bfloat16)
    out = ops.rms_norm(x, w, 1e-6)
    _close(out, ref.rms_norm(x.cpu(), w.cpu(), 1e-6), atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("d", [1024, 4096, 8192])
def test_fused_add_rmsnorm(d):
    torch.manual_seed(1)
    x = torch.randn(33, d, device=DEV, dtype=torch.bfloat16)
    r = torch.randn(33, d, device=DEV, dtype=torch.bfloat16)
    r_ref = (x.float().cpu() + r.float().cpu()).bfloat16()
    out, r2 = ops.fused_add_rms_norm(x, r, torch.ones(d, device=DEV, dtype=torch.bfloat16), 1e-5)
    _close(r2, r_ref, atol=1e-6)
    _close(out, ref.rms_norm(r_ref, torch.ones(d, dtype=torch.bfloat16), 1e-5), atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("T,F", [(1, 3072), (37, 3072), (256, 14336), (513, 14336)])
def test_silu_and_mul(T, F):
    x = torch.randn(T, 2 * F, device=DEV, dtype=torch.bfloat16)
    _close(ops.silu_and_mul(x), ref.silu_and_mul(x.cpu()), atol=2e-2, rtol=1e-2)


def _rand_cache(nb, hkv, bs, d=128, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    k = torch.randn(nb, hkv, bs, d, generator=g).bfloat16()
    v = torch.randn(nb, hkv, bs // 8, d, 8, generator=g).bfloat16()
    return k, v


@pytest.mark.parametrize("qk_norm", [True, False])
@pytest.mark.parametrize("hq,hkv", [(16, 8), (32, 8)])
@pytest.mark.parametrize("layout", ["random", "prefill"])
def test_qk_norm_rope_cache(qk_norm, hq, hkv, layout):
    torch.manual_seed(2)
    T, D, BS, NB = 45, 128, 32, 16
    qkv = torch.randn(T, (hq + 2 * hkv) * D, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), dtype=torch.int64)
    if layout == "random":
        slots = torch.randperm(NB * BS)[:T].to(torch.int64)
    else:  # two sequences' prefill chunks: complete 8-token V groups + ragged edges
        slots = torch.cat([torch.arange(3 * BS + 5, 3 * BS + 5 + 30),
                           torch.arange(9 * BS + 16, 9 * BS + 16 + 15)]).to(torch.int64)
    slots[3] = -1
    cs = ref.rope_cos_sin(4096, D, 1e6)
    qw = torch.randn(D).bfloat16() if qk_norm else None
    kw = torch.randn(D).bfloat16() if qk_norm else None
    kc, vc = torch.zeros(NB, hkv, BS, D).bfloat16(), torch.zeros(NB, hkv, BS // 8, D, 8).bfloat16()
    q_ref = torch.empty(T, hq, D).bfloat16()
    ref.qk_norm_rope_cache(qkv, q_ref, kc, vc, pos, slots, cs, qw, kw, hq, hkv, 1e-6)
    kg, vg = kc.zero_().to(DEV), vc.zero_().to(DEV)
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
    ref.qk_norm_rope_cache(qkv, q_ref, kc2, vc2, pos, slots, cs, qw, kw, hq, hkv, 1e-6)
    q_out = torch.empty(T, hq, D, device=DEV, dtype=torch.bfloat16)
    ops.qk_norm_rope_cache(qkv.to(DEV), q_out, kg, vg, pos.to(DEV), slots.to(DEV), cs.to(DEV),
                           None if qw is None else qw.to(DEV), None if kw is None else kw.to(DEV),
                           hq, hkv, 1e-6)
    _close(q_out, q_ref, atol=3e-2, rtol=2e-2)
    _close(kg, kc2, atol=3e-2, rtol=2e-2)
    _close(vg, vc2, atol=0)


def _setup_attn(seqs, hq, hkv, bs, seed=0):
    """seqs: list of (kv_len, q_len). Returns tensors on CPU."""
    g = torch.Generator().manual_seed(seed)
    D = 128
    nb_per = [math.ceil(kv / bs) for kv, _ in seqs]
    NB = sum(nb_per) + 3
    perm = torch.randperm(NB, generator=g)
    kc, vc = _rand_cache(NB, hkv, bs, D, seed)
    maxb = max(nb_per)
    bt = torch.zeros(len(seqs), maxb, dtype=torch.int32)
    i = 0
    for s, n in enumerate(nb_per):
        bt[s, :n] = perm[i:i + n].to(torch.int32)
        i += n
    q_start = torch.zeros(len(seqs) + 1, dtype=torch.int32)
    for s, (_, ql) in enumerate(seqs):
        q_start[s + 1] = q_start[s] + ql
    T = int(q_start[-1])
    q = torch.randn(T, hq, D, generator=g).bfloat16()
    seq_lens = torch.tensor([kv for kv, _ in seqs], dtype=torch.int32)
    return q, kc, vc, bt, seq_lens, q_start


def _tiles(seqs, G, rows=64):
    ts, tr = [], []
    for s, (_, ql) in enumerate(seqs):
        for r in range(0, ql * G, rows):
            ts.append(s)
            tr.append(r)
    return torch.tensor(ts, dtype=torch.int32), torch.tensor(tr, dtype=torch.int32)


@pytest.mark.parametrize("bs", [32, 64])
@pytest.mark.parametrize("hq,hkv", [(16, 8), (32, 8), (8, 8), (64, 8)])
@pytest.mark.parametrize("tile_rows", [128, 256])
def test_paged_attention_prefill(bs, hq, hkv, tile_rows):
    seqs = [(1, 1), (37, 37), (300, 300), (129, 64), (520, 7), (64, 1), (700, 650)]
    q, kc, vc, bt, sl, qs = _setup_attn(seqs, hq, hkv, bs, seed=bs + hq)
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q, kc, vc, bt, sl, qs, scale)
    ts, tr = _tiles(seqs, hq // hkv, tile_rows)
    out = torch.empty_like(q).to(DEV)
    ops.paged_attention_prefill(out, q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), sl.to(DEV),
                                qs.to(DEV), ts.to(DEV), tr.to(DEV), hq // hkv, scale,
                                tile_rows=tile_rows)
    _close(out, exp, atol=2e-2, rtol=2e-2)


# odd GQA groups (8/8, 24/8) take the full rotary-row loads, even ones the lane-pair share
@pytest.mark.parametrize("hq,hkv", [(16, 8), (32, 8), (8, 8), (24, 8)])
@pytest.mark.parametrize("qk_norm", [True, False])
@pytest.mark.parametrize("tile_rows", [128, 256])
def test_paged_attention_prefill_qprep(hq, hkv, qk_norm, tile_rows):
    """Prefill attention that norms + rotates its own q rows from the raw QKV projection
    (the serving prefill path) against the two-pass path: qk_norm_rope_cache writing every q
    row, then the kernel reading q.  Also: q_rows limits the standalone pass's q writes to the
    leading (decode) rows and leaves the others untouched."""
    seqs = [(1, 1), (37, 37), (300, 300), (129, 64), (520, 7), (700, 650)]
    _, kc, vc, bt, sl, qs = _setup_attn(seqs, hq, hkv, 32, seed=hq + tile_rows)
    G, D = hq // hkv, 128
    T = int(qs[-1])
    g = torch.Generator().manual_seed(7 + hq)
    qkv = (torch.randn(T, (hq + 2 * hkv) * D, generator=g) * 2.0).bfloat16().to(DEV)
    pos = torch.cat([torch.arange(kv - ql, kv) for kv, ql in seqs]).to(torch.int64).to(DEV)
    slots = torch.full((T,), -1, dtype=torch.int64, device=DEV)  # caches stay as built
    cs = ref.rope_cos_sin(1024, D, 1e6, device=DEV)
    qw = (torch.randn(D, generator=g) * 0.3 + 1.0).bfloat16().to(DEV) if qk_norm else None
    kw = (torch.randn(D, generator=g) * 0.3 + 1.0).bfloat16().to(DEV) if qk_norm else None
    kcd, vcd = kc.to(DEV), vc.to(DEV)
    q = torch.empty(T, hq, D, dtype=torch.bfloat16, device=DEV)
    ops.qk_norm_rope_cache(qkv, q, kcd, vcd, pos, slots, cs, qw, kw, hq, hkv, 1e-6, True)
    ts, tr = _tiles(seqs, G, tile_rows)
    args = (kcd, vcd, bt.to(DEV), sl.to(DEV), qs.to(DEV), ts.to(DEV), tr.to(DEV), G,
            1 / math.sqrt(D))
    exp = torch.empty_like(q)
    ops.paged_attention_prefill(exp, q, *args, tile_rows=tile_rows)
    out = torch.empty_like(q)
    ops.paged_attention_prefill(out, torch.empty_like(q), *args, tile_rows=tile_rows,
                                qprep=(qkv, pos, cs, qw, 1e-6))
    _close(out, exp, atol=1e-2, rtol=1e-2)
    # q_rows: only the first 5 tokens' q rows are written
    q2 = torch.full_like(q, 3.0)
    ops.qk_norm_rope_cache(qkv, q2, kcd, vcd, pos, slots, cs, qw, kw, hq, hkv, 1e-6, True,
                           q_rows=5)
    assert torch.equal(q2[:5], q[:5])
    assert bool((q2[5:] == 3.0).all())


@pytest.mark.parametrize("num_parts,part_size", [(1, 4096), (8, 256), (3, 512)])
@pytest.mark.parametrize("hq,hkv", [(16, 8), (64, 8), (32, 8)])
def test_paged_attention_decode(num_parts, part_size, hq, hkv):
    lens = [1, 31, 32, 33, 200, 777, 1500]
    if num_parts * part_size < max(lens):
        lens = [min(x, num_parts * part_size) for x in lens]
    seqs = [(kv, 1) for kv in lens]
    q, kc, vc, bt, sl, qs = _setup_attn(seqs, hq, hkv, 32, seed=num_parts)
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q, kc, vc, bt, sl, qs, scale)
    out = torch.empty_like(q).to(DEV)
    G = hq // hkv
    ws = ops.decode_workspace(len(seqs), hkv, G, num_parts, DEV)
    ops.paged_attention_decode(out, q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), sl.to(DEV), G,
                               scale, workspace=ws, num_parts=num_parts, part_size=part_size)
    _close(out, exp, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("hq,hkv", [(16, 8), (32, 8), (64, 8)])
@pytest.mark.parametrize("qk_norm", [True, False])
@pytest.mark.parametrize("num_parts,part_size", [(1, 4096), (3, 512)])
def test_paged_attention_decode_fused(hq, hkv, qk_norm, num_parts, part_size, lens=None):
    """Fused q/k-norm + RoPE + KV write + decode attention vs the reference pipeline."""
    lens = lens or [1, 31, 32, 33, 200, 777, 1500]
    seqs = [(kv, 1) for kv in lens]
    _, kc, vc, bt, sl, qs = _setup_attn(seqs, hq, hkv, 32, seed=hq + num_parts)
    B, D = len(lens), 128
    g = torch.Generator().manual_seed(11)
    qkv = torch.randn(B, (hq + 2 * hkv) * D, generator=g).bfloat16()
    pos = (sl - 1).to(torch.int64)
    slots = torch.tensor([int(bt[s, int(pos[s]) // 32]) * 32 + int(pos[s]) % 32
                          for s in range(B)], dtype=torch.int64)
    slots[2] = -1  # padding row: no cache write
    cs = ref.rope_cos_sin(max(4096, max(lens)), D, 1e6)
    qw = torch.randn(D, generator=g).bfloat16() if qk_norm else None
    kw = torch.randn(D, generator=g).bfloat16() if qk_norm else None
    kc_ref, vc_ref = kc.clone(), vc.clone()
    q_ref = torch.empty(B, hq, D).bfloat16()
    ref.qk_norm_rope_cache(qkv, q_ref, kc_ref, vc_ref, pos, slots, cs, qw, kw, hq, hkv, 1e-6)
    scale = 1 / math.sqrt(D)
    exp = ref.paged_attention(q_ref, kc_ref, vc_ref, bt, sl, qs, scale)
    kg, vg = kc.to(DEV), vc.to(DEV)
    out = torch.empty(B, hq, D, dtype=torch.bfloat16, device=DEV)
    G = hq // hkv
    ws = ops.decode_workspace(B, hkv, G, num_parts, DEV)
    ops.paged_attention_decode_fused(out, qkv.to(DEV), kg, vg, bt.to(DEV), sl.to(DEV),
                                     pos.to(DEV), slots.to(DEV), cs.to(DEV),
                                     None if qw is None else qw.to(DEV),
                                     None if kw is None else kw.to(DEV), G, scale, 1e-6,
                                     workspace=ws, num_parts=num_parts, part_size=part_size)
    _close(out, exp, atol=3e-2, rtol=3e-2)
    _close(kg, kc_ref, atol=3e-2, rtol=2e-2)
    _close(vg, vc_ref, atol=0)


def test_decode_attention_large_score_spike():
    """Force the online-softmax rescale branch: a single huge-score key late in the sequence."""
    seqs = [(900, 1)]
    q, kc, vc, bt, sl, qs = _setup_attn(seqs, 16, 8, 32, seed=5)
    b = int(bt[0, 27])
    ref.write_k(kc, b, 5, q[0, ::2, :] * 8)  # key 869 aligns with every q head of each kv head
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q, kc, vc, bt, sl, qs, scale)
    for parts, ps in [(1, 1024), (4, 256)]:
        out = torch.empty_like(q).to(DEV)
        ops.paged_attention_decode(out, q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), sl.to(DEV),
                                   2, scale, num_parts=parts, part_size=ps)
        _close(out, exp, atol=2e-2, rtol=2e-2)


def test_argmax_and_greedy_sample():
    torch.manual_seed(3)
    B, V = 9, 151936
    logits = torch.randn(B, V, device=DEV)
    logits[4, 77777] = 100.0
    exp = logits.argmax(-1)
    assert torch.equal(ops.argmax(logits), exp)
    assert torch.equal(ops.argmax(logits.bfloat16()), logits.bfloat16().float().argmax(-1))
    zeros = torch.zeros(B, device=DEV)
    tok, _ = ops.sample(logits, zeros, torch.zeros(B, dtype=torch.int32, device=DEV),
                        torch.ones(B, device=DEV), torch.arange(B, device=DEV),
                        torch.zeros(B, dtype=torch.int32, device=DEV))
    assert torch.equal(tok, exp)


@pytest.mark.parametrize("k,tp,scale", [(50, 1.0, 2.5), (0, 0.9, 2.5), (40, 0.8, 2.5),
                                        (2000, 0.5, 2.5), (1, 1.0, 2.5),
                                        # thresholds below the 256-key window under the max:
                                        # pass W cannot resolve them, passes A-C do
                                        (30000, 1.0, 0.3), (0, 0.9, 1.0), (40000, 0.9, 1.0)])
def test_sampling_filters_exact_sets_full_vocab(k, tp, scale):
    """Top-k / top-p on full-vocabulary bf16 rows (the window pass, or the distributed
    two-level threshold passes): every sampled token lies in the exact allowed set computed in
    fp32 from the same bf16 values (ties at the threshold included), over many (seed, step)
    draws."""
    torch.manual_seed(k + int(tp * 10))
    B, V, T = 16, 151936, 0.9
    base = (torch.randn(B, V) * scale).bfloat16()
    base[:, :7] = 9.0  # a tie group at the top
    logits = base.to(DEV)
    temp = torch.full((B,), T, device=DEV)
    tk = torch.full((B,), k, dtype=torch.int32, device=DEV)
    tpp = torch.full((B,), tp, device=DEV)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 7919
    allowed = []
    for r in range(B):
        z = base[r].float() / T
        keep = torch.ones(V, dtype=torch.bool)
        if 0 < k < V:
            kth = torch.topk(base[r].float(), k).values[-1]
            keep &= base[r].float() >= kth
        if 0 < tp < 1:
            p = torch.softmax(torch.where(keep, z, torch.tensor(-float("inf"))), -1)
            vals = base[r].float()
            order = torch.argsort(vals, descending=True)
            cum = torch.cumsum(p[order], 0)
            n = int((cum < tp - 1e-6).sum()) + 1
            thr = vals[order[n - 1]]
            keep &= vals >= thr
        allowed.append(keep)
    for step in range(24):
        steps = torch.full((B,), step, dtype=torch.int32, device=DEV)
        tok, lp = ops.sample(logits, temp, tk, tpp, seeds, steps)
        tok = tok.cpu()
        for r in range(B):
            assert bool(allowed[r][tok[r]]), (r, step, int(tok[r]))
    # one-token sets are deterministic
    if k == 1:
        assert all(int(allowed[r].sum()) >= 1 for r in range(B))


def test_sampling_distribution_topk_topp():
    torch.manual_seed(4)
    V, N = 64, 4000
    base = torch.randn(V) * 2
    logits = base.expand(N, V).contiguous().to(DEV)
    temp = torch.full((N,), 0.8, device=DEV)
    seeds = torch.full((N,), 1234, dtype=torch.int64, device=DEV)
    steps = torch.arange(N, dtype=torch.int32, device=DEV)
    # plain temperature
    tok, lp = ops.sample(logits, temp, torch.zeros(N, dtype=torch.int32, device=DEV),
                         torch.ones(N, device=DEV), seeds, steps)
    p = torch.softmax(base / 0.8, -1)
    freq = torch.bincount(tok.cpu(), minlength=V).float() / N
    assert (freq - p).abs().max() < 0.03
    _close(lp, torch.log(p[tok.cpu()]), atol=1e-3)
    # top-k
    k = 5
    tok, _ = ops.sample(logits, temp, torch.full((N,), k, dtype=torch.int32, device=DEV),
                        torch.ones(N, device=DEV), seeds, steps)
    top = set(torch.topk(base, k).indices.tolist())
    assert set(tok.cpu().tolist()) <= top
    assert len(set(tok.cpu().tolist())) == k
    # top-p
    tp = 0.7
    tok, _ = ops.sample(logits, temp, torch.zeros(N, dtype=torch.int32, device=DEV),
                        torch.full((N,), tp, device=DEV), seeds, steps)
    sp, si = p.sort(descending=True)
    n = int((sp.cumsum(0) < tp).sum()) + 1
    nucleus = set(si[:n].tolist())
    assert set(tok.cpu().tolist()) <= nucleus
    # reproducible per (seed, step)
    tok2, _ = ops.sample(logits, temp, torch.zeros(N, dtype=torch.int32, device=DEV),
                         torch.full((N,), tp, device=DEV), seeds, steps)
    assert torch.equal(tok, tok2)


@pytest.mark.parametrize("B,dtype,aligned", [(256, torch.bfloat16, True),
                                             (8, torch.bfloat16, True),
                                             (64, torch.float32, True),
                                             (64, torch.bfloat16, False)])
def test_sampling_distribution_full_vocab_tiles(B, dtype, aligned):
    """Plain temperature draws on full-vocabulary rows: the row's chunk, then the tile inside
    it (published tile masses), then one 2048-element rescan.  Hot tokens sit on tile and chunk
    boundaries; their frequencies over 4096 draws match the fp32 softmax, and the log-probs
    match.  Unaligned rows (a view one element in) take the scalar path."""
    torch.manual_seed(B)
    V = 151936
    base = torch.randn(V) * 0.5
    hot = {5: 12.0, 2047: 13.0, 2048: 11.5, 40000: 12.5, 75967: 13.0, 75968: 12.0,
           151935: 11.0, 151930: 10.5}
    for i, v in hot.items():
        base[i] = v
    vals = base.to(dtype).float()
    T = 1.0
    p = torch.softmax(vals / T, -1)
    rows = vals.to(dtype).expand(B, V)
    if aligned:
        logits = rows.contiguous().to(DEV)
    else:
        big = torch.zeros(B, V + 1, dtype=dtype)
        big[:, 1:] = rows
        logits = big.to(DEV)[:, 1:]
    temp = torch.full((B,), T, device=DEV)
    tk = torch.zeros(B, dtype=torch.int32, device=DEV)
    tp = torch.ones(B, device=DEV)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 104729
    toks, lps = [], []
    for step in range(4096 // B):
        steps = torch.full((B,), step, dtype=torch.int32, device=DEV)
        tok, lp = ops.sample(logits, temp, tk, tp, seeds, steps, filtered=False)
        toks.append(tok.cpu())
        lps.append(lp.cpu())
    tok = torch.cat(toks)
    lp = torch.cat(lps)
    n = tok.numel()
    assert int(tok.min()) >= 0 and int(tok.max()) < V
    for i in hot:
        f = float((tok == i).sum()) / n
        assert abs(f - float(p[i])) < 0.03, (i, f, float(p[i]))
    rest = 1.0 - sum(float(p[i]) for i in hot)
    f_rest = float((~torch.isin(tok, torch.tensor(list(hot)))).sum()) / n
    assert abs(f_rest - rest) < 0.03, (f_rest, rest)
    _close(lp, torch.log(p[tok]), atol=2e-3)


@pytest.mark.parametrize("k,tp", [(0, 1.0), (50, 1.0), (0, 0.9)])
def test_sampling_fully_masked_row_stays_in_range(k, tp):
    """A row whose every logit is -inf (a fully masked vocabulary) must not send the draw to a
    chunk / tile index of -1: every token comes back inside [0, V), and the other rows of the
    batch are unaffected (their greedy-equivalent hot token wins)."""
    B, V = 4, 151936
    logits = torch.full((B, V), -30.0)
    for r in range(B):
        logits[r, 1000 * (r + 1)] = 30.0
    logits[2] = -float("inf")
    x = logits.to(torch.bfloat16).to(DEV)
    temp = torch.ones(B, device=DEV)
    tk = torch.full((B,), k, dtype=torch.int32, device=DEV)
    tpp = torch.full((B,), tp, device=DEV)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV)
    steps = torch.zeros(B, dtype=torch.int32, device=DEV)
    tok, _ = ops.sample(x, temp, tk, tpp, seeds, steps, filtered=k > 0 or tp < 1.0)
    tok = tok.cpu()
    assert int(tok.min()) >= 0 and int(tok.max()) < V
    for r in (0, 1, 3):
        assert int(tok[r]) == 1000 * (r + 1)


@pytest.mark.parametrize("B,V", [(12, 128256), (300, 128256), (40, 32000)])
def test_sampling_mixed_rows_one_batch(B, V):
    """One launch whose rows mix every mode the server sends: greedy (T = 0), plain temperature,
    top-k, top-p, top-k + top-p and k = 1, at Llama-3's and Llama-2's vocabularies (a partial last
    tile) and past 256 rows.  Per-row state (resolved flags, thresholds) must not leak between
    rows: greedy rows return the argmax, filtered rows stay inside their exact allowed set,
    every token is in [0, V)."""
    torch.manual_seed(B + V)
    base = (torch.randn(B, V) * 2.0).bfloat16()
    modes = [(0.0, 0, 1.0), (1.0, 0, 1.0), (0.8, 40, 1.0), (1.0, 0, 0.9), (0.7, 200, 0.8),
             (1.0, 1, 1.0)]
    temp, tk, tpp = [], [], []
    for r in range(B):
        t, k, p = modes[r % len(modes)]
        temp.append(t)
        tk.append(k)
        tpp.append(p)
    allowed = []
    for r in range(B):
        vals = base[r].float()
        keep = torch.ones(V, dtype=torch.bool)
        if temp[r] == 0.0:
            keep = torch.zeros(V, dtype=torch.bool)
            keep[vals.argmax()] = True
        else:
            if 0 < tk[r] < V:
                keep &= vals >= torch.topk(vals, tk[r]).values[-1]
            if tpp[r] < 1.0:
                z = torch.where(keep, vals / temp[r], torch.tensor(-float("inf")))
                pr = torch.softmax(z, -1)
                order = torch.argsort(vals, descending=True)
                cum = torch.cumsum(pr[order], 0)
                n = int((cum < tpp[r] - 1e-6).sum()) + 1
                keep &= vals >= vals[order[n - 1]]
        allowed.append(keep)
    logits = base.to(DEV)
    args = (torch.tensor(temp, device=DEV), torch.tensor(tk, dtype=torch.int32, device=DEV),
            torch.tensor(tpp, device=DEV), torch.arange(B, dtype=torch.int64, device=DEV) * 31)
    for step in range(6):
        steps = torch.full((B,), step, dtype=torch.int32, device=DEV)
        tok, _ = ops.sample(logits, args[0], args[1], args[2], args[3], steps)
        tok = tok.cpu()
        assert int(tok.min()) >= 0 and int(tok.max()) < V
        for r in range(B):
            assert bool(allowed[r][tok[r]]), (r, step, temp[r], tk[r], tpp[r], int(tok[r]))


@pytest.mark.parametrize("T,d", [(1, 1024), (37, 1024), (256, 4096), (5, 8)])
def test_embedding_prep_matches_reference(T, d):
    """Decode prologue in one launch: embedding rows, rows * ln, row sums of squares, and the
    accumulator buffer zeroed -- against the fp32 reference of the three separate ops."""
    g = torch.Generator().manual_seed(T + d)
    table = (torch.randn(300, d, generator=g) * 0.5).bfloat16()
    ln = torch.randn(d, generator=g).bfloat16()
    ids = torch.randint(0, 400, (T,), generator=g)  # ids >= 300 fall outside this shard
    x = ref.embedding(ids, table, 0, 300)
    res = torch.empty(T, d, dtype=torch.bfloat16, device=DEV)
    a = torch.empty_like(res)
    ss = torch.full((T,), 7.0, device=DEV)
    z = torch.full((3, T), 5.0, device=DEV)
    ops.embedding_prep(ids.to(DEV), table.to(DEV), ln.to(DEV), res, a, ss, z, 0, 300)
    _close(res, x, atol=0)
    _close(a, (x.float() * ln.float()).bfloat16(), atol=1e-2, rtol=1e-2)
    _close(ss, x.float().pow(2).sum(-1), atol=1e-3, rtol=1e-4)
    assert float(z.abs().max()) == 0.0


def test_embedding_vocab_parallel():
    table = torch.randn(1000, 1024, dtype=torch.bfloat16)
    ids = torch.tensor([0, 5, 999, 1500, 250], dtype=torch.int64)
    exp = ref.embedding(ids, table, 0, 1000)
    out = ops.embedding(ids.to(DEV), table.to(DEV))
    _close(out, exp, atol=0)
    exp2 = ref.embedding(ids, table[200:600], 200, 600)
    out2 = ops.embedding(ids.to(DEV), table[200:600].contiguous().to(DEV), vocab_start=200,
                         vocab_end=600)
    _close(out2, exp2, atol=0)


@pytest.mark.parametrize("T,E,K,d", [(1, 8, 2, 4096), (37, 8, 2, 4096), (128, 8, 2, 4096),
                                     (64, 16, 4, 1024), (5, 3, 1, 256)])
def test_moe_router_topk_fused(T, E, K, d):
    """Router GEMM + softmax + top-k in one launch vs fp32 logits rounded to bf16 + reference."""
    g = torch.Generator().manual_seed(T + E)
    h = (torch.randn(T, d, generator=g) * 0.5).bfloat16()
    router = (torch.randn(E, d, generator=g) * 0.05).bfloat16()
    logits = (h.float() @ router.float().t()).bfloat16()
    rw, rid = ref.moe_topk_softmax(logits, K)
    w = torch.empty(T, K, dtype=torch.float32, device=DEV)
    ids = torch.empty(T, K, dtype=torch.int32, device=DEV)
    torch.ops.akap.moe_router_topk(h.to(DEV), router.to(DEV), w, ids, True)
    # bf16 logits tie often at E = 8: compare the selected (expert, weight) sets, not the order
    # among equal logits (ours: lowest id first; torch.topk: unspecified)
    oi, o = ids.cpu().long().sort(dim=-1)
    ri, r = rid.long().sort(dim=-1)
    assert torch.equal(oi, ri)
    _close(w.cpu().gather(1, o), rw.gather(1, r), atol=1e-3)
    w2, ids2 = ops.moe_router_topk(h.to(DEV), router.to(DEV), K)  # the dispatching wrapper
    assert torch.equal(ids2.cpu(), ids.cpu())


@pytest.mark.parametrize("T,E,K", [(256, 128, 8), (37, 256, 8), (1000, 64, 4), (5, 48, 1)])
def test_moe_topk_softmax_many_experts(T, E, K):
    """The wave-per-token routing kernel (E > 32) vs the fp32 reference: same experts, same
    weights; renormalised and raw."""
    g = torch.Generator().manual_seed(T + E)
    # distinct logits per row (no bf16 ties at the K-th boundary): a random permutation of an
    # evenly spaced grid in [-1, 1), exactly representable in bf16
    perm = torch.argsort(torch.rand(T, E, generator=g), dim=-1).float()
    logits = ((perm - E / 2) * (2.0 / E)).bfloat16()
    assert all(len(set(r.tolist())) == E for r in logits.float())
    for renorm in (True, False):
        w, ids = ops.moe_topk_softmax(logits.to(DEV), K, renormalize=renorm)
        rw, rid = ref.moe_topk_softmax(logits, K, renorm)
        oi, o = ids.cpu().long().sort(dim=-1)
        ri, r = rid.long().sort(dim=-1)
        assert torch.equal(oi, ri)
        _close(w.cpu().gather(1, o), rw.gather(1, r), atol=1e-4)


def test_moe_routing():
    torch.manual_seed(6)
    T, E, K = 300, 8, 2
    logits = torch.randn(T, E, dtype=torch.bfloat16)
    w, ids = ops.moe_topk_softmax(logits.to(DEV), K)
    rw, rid = ref.moe_topk_softmax(logits, K)
    assert torch.equal(ids.cpu(), rid)
    _close(w, rw, atol=1e-4)
    s, off, npad = ops.moe_align(ids, E, 16)
    off = off.cpu()
    s = s.cpu()
    flat = ids.cpu().reshape(-1)
    for e in range(E):
        seg = s[off[e]:off[e + 1]]
        real = seg[seg < T * K]
        assert set(real.tolist()) == set((flat == e).nonzero().flatten().tolist())
        assert (off[e + 1] - off[e]) % 16 == 0
    assert int(npad) == int(off[-1])


def test_moe_align_inv_and_tiles():
    torch.manual_seed(9)
    T, E, K = 77, 8, 2
    ids = torch.randint(0, E, (T, K), dtype=torch.int32, device=DEV)
    n = T * K
    cap = ops.moe_capacity(n, E, 64)
    inv = torch.empty(n, dtype=torch.int32, device=DEV)
    te = torch.empty(cap // 64, dtype=torch.int32, device=DEV)
    s, off, npad = ops.moe_align(ids, E, 64, inv=inv, tile_expert=te)
    s, off, inv, te = s.cpu(), off.cpu(), inv.cpu(), te.cpu()
    assert torch.equal(s[inv.long()], torch.arange(n, dtype=torch.int32))
    for t in range(cap // 64):
        if t * 64 >= int(off[-1]):
            assert int(te[t]) == -1
        else:
            e = int(te[t])
            assert off[e] <= t * 64 < off[e + 1]


@pytest.mark.parametrize("T,E,K,d,F", [(1, 8, 2, 256, 512), (37, 8, 2, 512, 384),
                                       (256, 8, 2, 256, 256), (64, 16, 4, 128, 192)])
def test_fused_moe(T, E, K, d, F):
    torch.manual_seed(T + E)
    h = torch.randn(T, d, dtype=torch.bfloat16)
    w13 = torch.randn(E, 2 * F, d, dtype=torch.bfloat16) * d ** -0.5
    w2 = torch.randn(E, d, F, dtype=torch.bfloat16) * F ** -0.5
    logits = torch.randn(T, E, dtype=torch.bfloat16)
    w, ids = ref.moe_topk_softmax(logits, K)
    exp = ref.fused_moe(h, w13, w2, w, ids)
    out = ops.fused_moe(h.to(DEV), w13.to(DEV), w2.to(DEV), w.to(DEV), ids.to(DEV))
    _close(out, exp, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("T", [64, 1024])
def test_moe_block_tp_paths_match_reference(T):
    """TP-mode MoE block: decode sizes on fused_moe, prefill sizes (T >= 512) on the
    torch._grouped_mm path -- both against the fp32 reference of the same routing."""
    from aws_k8s_ansible_provisioner_amd.models.config import get_config
    from aws_k8s_ansible_provisioner_amd.models.moe import MoEBlock
    from aws_k8s_ansible_provisioner_amd.parallel.state import ParallelState

    cfg = get_config("tiny-mixtral8")
    blk = MoEBlock(cfg, ParallelState(rank=0, world_size=1, tp_size=1), DEV, torch.bfloat16,
                   torch.Generator().manual_seed(0), full_then_shard=False, mode="tp")
    torch.manual_seed(T)
    h = torch.randn(T, cfg.hidden_size, dtype=torch.bfloat16, device=DEV)
    out = blk.forward(h)
    w, ids = ops.moe_router_topk(h, blk.router, blk.K, renormalize=True)
    exp = ref.fused_moe(h.cpu(), blk.w13.cpu(), blk.w2.cpu(), w.cpu(), ids.cpu())
    _close(out, exp, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("R", [1536, 4096])
def test_moe_expert_rows_skip_empty_slots_gpu(R):
    """The EP fixed-dispatch receive rows at prefill sizes on the grouped GEMM (pgemm or
    torch._grouped_mm): empty slots (id -1) fall in a dummy group past the last offset; real
    rows match the fp32 reference."""
    from aws_k8s_ansible_provisioner_amd.models.config import get_config
    from aws_k8s_ansible_provisioner_amd.models.moe import MoEBlock
    from aws_k8s_ansible_provisioner_amd.parallel.state import ParallelState

    cfg = get_config("tiny-mixtral8")
    blk = MoEBlock(cfg, ParallelState(rank=0, world_size=1, tp_size=1), DEV, torch.bfloat16,
                   torch.Generator().manual_seed(0), full_then_shard=False, mode="tp")
    torch.manual_seed(R)
    x = torch.randn(R, cfg.hidden_size, dtype=torch.bfloat16)
    e = torch.randint(0, blk.e_local, (R,))
    e[torch.rand(R) < 0.5] = -1
    y = blk._expert_rows(x.to(DEV), e.to(torch.int32).to(DEV)).cpu()
    real = e >= 0
    one = torch.ones(R, 1)
    exp = ref.fused_moe(x[real], blk.w13.cpu(), blk.w2.cpu(), one[real],
                        e[real].view(-1, 1).to(torch.int32))
    _close(y[real], exp, atol=3e-2, rtol=3e-2)


def test_fused_moe_graph_capture():
    torch.manual_seed(3)
    T, E, K, d, F = 48, 8, 2, 256, 256
    h = torch.randn(T, d, dtype=torch.bfloat16, device=DEV)
    w13 = torch.randn(E, 2 * F, d, dtype=torch.bfloat16, device=DEV) * 0.06
    w2 = torch.randn(E, d, F, dtype=torch.bfloat16, device=DEV) * 0.06
    logits = torch.randn(T, E, dtype=torch.bfloat16, device=DEV)
    out = torch.empty(T, d, dtype=torch.bfloat16, device=DEV)

    def run():
        w, ids = ops.moe_topk_softmax(logits, K)
        ops.fused_moe(h, w13, w2, w, ids, out=out)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run()
    logits.copy_(torch.randn(T, E, dtype=torch.bfloat16, device=DEV))
    g.replay()
    torch.cuda.synchronize()
    w, ids = ref.moe_topk_softmax(logits.cpu(), K)
    exp = ref.fused_moe(h.cpu(), w13.cpu(), w2.cpu(), w, ids)
    _close(out, exp, atol=3e-2, rtol=3e-2)


def test_kv_gather_scatter_roundtrip():
    planes, NB = 6, 20
    cache = torch.randn(planes, NB, 8, 32, 128, dtype=torch.bfloat16, device=DEV)
    ids = torch.tensor([3, 17, 0, 9], dtype=torch.int32, device=DEV)
    buf = ops.kv_gather(cache, ids)
    assert torch.equal(buf.view(planes, 4, -1), cache.view(planes, NB, -1)[:, ids.long()])
    dst = torch.zeros_like(cache)
    ids2 = torch.tensor([1, 2, 5, 19], dtype=torch.int32, device=DEV)
    ops.kv_scatter(buf, dst, ids2)
    assert torch.equal(dst.view(planes, NB, -1)[:, ids2.long()], buf.view(planes, 4, -1))


@pytest.mark.parametrize("M", [1, 7, 64, 100, 256, 512])
@pytest.mark.parametrize("N,K", [(4096, 1024), (1024, 2048), (6144, 1024), (1024, 3072),
                                 (1000, 520), (64, 64)])
@pytest.mark.parametrize("inlaunch", [False, True])
def test_decode_gemm(M, N, K, inlaunch):
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    ref_ = (x.float() @ w.float().t())
    s = ops.gemm_splitk(M, N, K)
    ws = torch.empty(max(1, s * M * N), device=DEV, dtype=torch.float32)
    cnt = ops.gemm_counters(x.device) if inlaunch else None
    for _ in range(3):  # repeated calls: the in-launch tickets must re-arm
        y = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
        torch.ops.akap.gemm(y, x, w, ws, s, cnt)
        err = (y.float() - ref_).abs().max().item()
        assert err <= 2e-2 * ref_.abs().max().item() + 1e-2, err
    if cnt is not None:
        assert int(cnt.abs().sum()) == 0  # every ticket re-armed


def test_decode_gemm_strided_input():
    x = torch.randn(64, 2048, device=DEV, dtype=torch.bfloat16)[:, :1024]
    w = torch.randn(512, 1024, device=DEV, dtype=torch.bfloat16) * 0.05
    ref_ = x.float() @ w.float().t()
    y = torch.empty(64, 512, device=DEV, dtype=torch.bfloat16)
    torch.ops.akap.gemm(y, x, w, torch.empty(1, device=DEV), 1)
    assert (y.float() - ref_).abs().max().item() < 3e-2 * ref_.abs().max().item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_apply_penalties(dtype):
    torch.manual_seed(12)
    B, V = 5, 1000
    logits = (torch.randn(B, V) * 3).to(dtype)
    rows = torch.tensor([0, 0, 1, 3, 3, 3, 4], dtype=torch.int32)
    toks = torch.tensor([3, 999, 3, 0, 1, 500, 7], dtype=torch.int32)
    counts = torch.tensor([2, 0, 1, 5, 0, 1, 3], dtype=torch.int32)
    pres = torch.tensor([0.5, 0.0, 1.0, 0.2, 0.0])
    freq = torch.tensor([0.1, 0.0, 0.3, 0.7, 0.0])
    rep = torch.tensor([1.3, 1.0, 1.0, 2.0, 1.1])
    exp = ref.apply_penalties(logits.float(), rows, toks, counts, pres, freq, rep)
    got = logits.to(DEV)
    ops.apply_penalties(got, rows.to(DEV), toks.to(DEV), counts.to(DEV), pres.to(DEV),
                        freq.to(DEV), rep.to(DEV))
    _close(got, exp, atol=5e-2 if dtype == torch.bfloat16 else 1e-5, rtol=1e-2)


def test_greedy_logprobs():
    torch.manual_seed(13)
    B, V = 6, 151936
    logits = torch.randn(B, V, device=DEV).bfloat16()
    z = torch.zeros(B, device=DEV)
    tok, lp = ops.sample(logits, z, torch.zeros(B, dtype=torch.int32, device=DEV),
                         torch.ones(B, device=DEV), torch.arange(B, device=DEV),
                         torch.zeros(B, dtype=torch.int32, device=DEV), greedy_logprobs=True)
    ls = torch.log_softmax(logits.float(), -1)
    exp = ls.gather(1, tok.view(-1, 1)).view(-1)
    assert torch.equal(tok, logits.float().argmax(-1))
    _close(lp, exp, atol=2e-3)


def test_gemm_tuner_plan_is_used_and_correct():
    from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner

    torch.manual_seed(21)
    ws = [torch.randn(1024, 3072, device=DEV, dtype=torch.bfloat16) * 0.02 for _ in range(4)]
    choice = gemm_tuner.tune(128, ws)
    assert choice[0] in ("torch", "hip", "dgemm", "wgemm")
    assert gemm_tuner.lookup(128, 1024, 3072) == choice
    x = torch.randn(128, 3072, device=DEV, dtype=torch.bfloat16)
    y = ops.linear(x, ws[1])
    ref_ = x.float() @ ws[1].float().t()
    assert (y.float() - ref_).abs().max().item() <= 2e-2 * ref_.abs().max().item() + 1e-2
    # force the MFMA path through the plan and check it too
    for forced in (("hip", 4), ("dgemm", 4, 2), ("dgemm", 1, 4), ("dgemm", 1, 1, 0, 0, False, 16),
                   ("dgemm", 1, 1, 0, 0, False, 32), ("wgemm",)):
        gemm_tuner.plan()[(128, 1024, 3072)] = forced
        y2 = ops.linear(x, ws[1])
        assert (y2.float() - ref_).abs().max().item() <= 2e-2 * ref_.abs().max().item() + 1e-2
    gemm_tuner.plan().pop((128, 1024, 3072))



def _to_fp8_cache(kc, vc):
    """bf16 test caches -> uint8 e4m3 caches (same values the kernels will read)."""
    f = lambda t: t.float().clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)  # noqa
    return f(kc), f(vc)


@pytest.mark.parametrize("hq,hkv", [(16, 8), (32, 8)])
@pytest.mark.parametrize("layout", ["random", "prefill"])
def test_qk_norm_rope_cache_fp8(hq, hkv, layout):
    torch.manual_seed(31)
    T, D, BS, NB = 45, 128, 32, 16
    qkv = torch.randn(T, (hq + 2 * hkv) * D, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), dtype=torch.int64)
    slots = (torch.randperm(NB * BS)[:T] if layout == "random" else
             torch.cat([torch.arange(3 * BS + 5, 3 * BS + 35), torch.arange(9 * BS + 16,
                                                                          9 * BS + 31)]))
    slots = slots.to(torch.int64)
    cs = ref.rope_cos_sin(4096, D, 1e6)
    qw, kw = torch.randn(D).bfloat16(), torch.randn(D).bfloat16()
    kc = torch.zeros(NB, hkv, BS, D, dtype=torch.uint8)
    vc = torch.zeros(NB, hkv, BS // 8, D, 8, dtype=torch.uint8)
    q_ref = torch.empty(T, hq, D).bfloat16()
    ref.qk_norm_rope_cache(qkv, q_ref, kc, vc, pos, slots, cs, qw, kw, hq, hkv, 1e-6)
    kg, vg = torch.zeros_like(kc).to(DEV), torch.zeros_like(vc).to(DEV)
    q_out = torch.empty(T, hq, D, device=DEV, dtype=torch.bfloat16)
    ops.qk_norm_rope_cache(qkv.to(DEV), q_out, kg, vg, pos.to(DEV), slots.to(DEV), cs.to(DEV),
                           qw.to(DEV), kw.to(DEV), hq, hkv, 1e-6)
    dq = lambda t: t.cpu().view(torch.float8_e4m3fn).float()  # noqa
    # K passes through fp32 norm+rope on both sides: allow one fp8 ulp on rare ties
    _close(dq(kg), dq(kc), atol=1e-2, rtol=0.13)
    assert torch.equal(vg.cpu(), vc)  # V is exact: bf16 -> e4m3 on both sides


@pytest.mark.parametrize("num_parts,part_size", [(1, 4096), (3, 512)])
@pytest.mark.parametrize("fused", [False, True])
def test_paged_attention_decode_fp8(num_parts, part_size, fused):
    lens = [1, 31, 33, 200, 777, 1500]
    seqs = [(kv, 1) for kv in lens]
    hq, hkv = 16, 8
    q, kc, vc, bt, sl, qs = _setup_attn(seqs, hq, hkv, 32, seed=41)
    kc8, vc8 = _to_fp8_cache(kc, vc)
    scale = 1 / math.sqrt(128)
    B, G = len(lens), hq // hkv
    ws = ops.decode_workspace(B, hkv, G, num_parts, DEV)
    out = torch.empty(B, hq, 128, dtype=torch.bfloat16, device=DEV)
    if not fused:
        exp = ref.paged_attention(q, kc8, vc8, bt, sl, qs, scale)
        ops.paged_attention_decode(out, q.to(DEV), kc8.to(DEV), vc8.to(DEV), bt.to(DEV),
                                   sl.to(DEV), G, scale, workspace=ws, num_parts=num_parts,
                                   part_size=part_size)
        _close(out, exp, atol=3e-2, rtol=3e-2)
        return
    g = torch.Generator().manual_seed(5)
    qkv = torch.randn(B, (hq + 2 * hkv) * 128, generator=g).bfloat16()
    pos = (sl - 1).to(torch.int64)
    slots = torch.tensor([int(bt[s, int(pos[s]) // 32]) * 32 + int(pos[s]) % 32
                          for s in range(B)], dtype=torch.int64)
    slots[1] = -1  # padding row: no cache write, attends what the cache holds
    cs = ref.rope_cos_sin(4096, 128, 1e6)
    kr, vr = kc8.clone(), vc8.clone()
    q_ref = torch.empty(B, hq, 128).bfloat16()
    ref.qk_norm_rope_cache(qkv, q_ref, kr, vr, pos, slots, cs, None, None, hq, hkv, 1e-6)
    exp = ref.paged_attention(q_ref, kr, vr, bt, sl, qs, scale)
    kg, vg = kc8.to(DEV), vc8.to(DEV)
    ops.paged_attention_decode_fused(out, qkv.to(DEV), kg, vg, bt.to(DEV), sl.to(DEV),
                                     pos.to(DEV), slots.to(DEV), cs.to(DEV), None, None, G,
                                     scale, 1e-6, workspace=ws, num_parts=num_parts,
                                     part_size=part_size)
    _close(out, exp, atol=4e-2, rtol=4e-2)
    dq = lambda t: t.cpu().view(torch.float8_e4m3fn).float()  # noqa: E731
    _close(dq(kg), dq(kr), atol=1e-2, rtol=0.13)
    assert torch.equal(vg.cpu(), vr)  # the new token's V group is stored back whole


@pytest.mark.parametrize("tile_rows", [128])
def test_paged_attention_prefill_fp8(tile_rows):
    seqs = [(1, 1), (37, 37), (300, 300), (129, 64), (700, 650)]
    hq, hkv = 16, 8
    q, kc, vc, bt, sl, qs = _setup_attn(seqs, hq, hkv, 32, seed=43)
    kc8, vc8 = _to_fp8_cache(kc, vc)
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q, kc8, vc8, bt, sl, qs, scale)
    ts, tr = _tiles(seqs, hq // hkv, tile_rows)
    out = torch.empty_like(q).to(DEV)
    ops.paged_attention_prefill(out, q.to(DEV), kc8.to(DEV), vc8.to(DEV), bt.to(DEV), sl.to(DEV),
                                qs.to(DEV), ts.to(DEV), tr.to(DEV), hq // hkv, scale,
                                tile_rows=tile_rows)
    _close(out, exp, atol=2e-2, rtol=2e-2)


def test_paged_attention_prefill_qprep_fp8():
    """The register-staged fp8-cache prefill kernel with its own q norm + RoPE against the same
    kernel reading the q rows the standalone pass wrote."""
    seqs = [(1, 1), (37, 37), (300, 300), (129, 64), (700, 650)]
    hq, hkv, D = 16, 8, 128
    _, kc, vc, bt, sl, qs = _setup_attn(seqs, hq, hkv, 32, seed=44)
    kc8, vc8 = _to_fp8_cache(kc, vc)
    kcd, vcd = kc8.to(DEV), vc8.to(DEV)
    T = int(qs[-1])
    g = torch.Generator().manual_seed(45)
    qkv = (torch.randn(T, (hq + 2 * hkv) * D, generator=g) * 2.0).bfloat16().to(DEV)
    pos = torch.cat([torch.arange(kv - ql, kv) for kv, ql in seqs]).to(torch.int64).to(DEV)
    slots = torch.full((T,), -1, dtype=torch.int64, device=DEV)
    cs = ref.rope_cos_sin(1024, D, 1e6, device=DEV)
    qw = (torch.randn(D, generator=g) * 0.3 + 1.0).bfloat16().to(DEV)
    q = torch.empty(T, hq, D, dtype=torch.bfloat16, device=DEV)
    ops.qk_norm_rope_cache(qkv, q, kcd, vcd, pos, slots, cs, qw, qw, hq, hkv, 1e-6, True)
    ts, tr = _tiles(seqs, hq // hkv, 128)
    args = (kcd, vcd, bt.to(DEV), sl.to(DEV), qs.to(DEV), ts.to(DEV), tr.to(DEV), hq // hkv,
            1 / math.sqrt(D))
    exp = torch.empty_like(q)
    ops.paged_attention_prefill(exp, q, *args, tile_rows=128)
    out = torch.empty_like(q)
    ops.paged_attention_prefill(out, torch.empty_like(q), *args, tile_rows=128,
                                qprep=(qkv, pos, cs, qw, 1e-6))
    _close(out, exp, atol=1e-2, rtol=1e-2)


def _dgemm_ref(pro, x, w, r, ln, eps):
    """fp32 reference of the fused decode GEMM's prologue + GEMM (+ residual out)."""
    x, w = x.float().cpu(), w.float().cpu()
    s = None
    if pro == ops.PRO_ADDNORM:
        s = (x + r.float().cpu()).to(torch.bfloat16)
        a = ref.rms_norm(s, ln.cpu(), eps).float()
    elif pro == ops.PRO_SILU:
        a = ref.silu_and_mul(x.to(torch.bfloat16)).float()
    else:
        a = x
    return a @ w.t(), s


@pytest.mark.parametrize("pro", [0, 1, 2])
@pytest.mark.parametrize("M,N,K", [(1, 256, 1024), (37, 1024, 2048), (256, 4096, 1024),
                                   (130, 3072, 512)])
@pytest.mark.parametrize("splitk,pf", [(1, 1), (1, 2), (2, 4), (4, 1), (8, 2)])
def test_fused_decode_gemm(pro, M, N, K, splitk, pf):
    if not ops.dgemm_supported(M, N, K, splitk, pf):
        pytest.skip("unsupported split/prefetch for this K")
    torch.manual_seed(M * 7 + N + pro)
    eps = 1e-6
    x = torch.randn(M, 2 * K if pro == ops.PRO_SILU else K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    r = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    ln = torch.rand(K, device=DEV, dtype=torch.bfloat16) + 0.5
    rout = torch.full_like(r, float("nan"))
    y = ops.dgemm(x, w, pro, splitk, pf, residual=r, residual_out=rout, ln=ln, eps=eps)
    torch.cuda.synchronize()
    want, s = _dgemm_ref(pro, x, w, r, ln, eps)
    scale = want.abs().max().item()
    _close(y, want, atol=2e-2 * scale)
    if pro == ops.PRO_ADDNORM:
        _close(rout, s, atol=0.0)


def test_fused_decode_gemm_in_graph():
    """Graph-captured split-K fused GEMM replays to the same result as eager."""
    torch.manual_seed(3)
    M, N, K = 64, 2048, 1024
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    r = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    rout = torch.empty_like(r)
    ln = torch.rand(K, device=DEV, dtype=torch.bfloat16) + 0.5
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    eager = ops.dgemm(x, w, ops.PRO_ADDNORM, 4, 2, residual=r, residual_out=rout, ln=ln).clone()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.dgemm(x, w, ops.PRO_ADDNORM, 4, 2, residual=r, residual_out=rout, ln=ln)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        y = ops.dgemm(x, w, ops.PRO_ADDNORM, 4, 2, residual=r, residual_out=rout, ln=ln)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y, eager)


@pytest.mark.parametrize("ring", ["shallow", "deep", "deep-inlaunch", "shallow-inlaunch",
                                  "rows128", "rows128-inlaunch", "rows256", "rows256-inlaunch",
                                  "rows256deep", "rows256deep-inlaunch"])
@pytest.mark.parametrize("bn", [64, 128])
@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("M,N,K,splitk", [(1, 256, 1024, 1), (37, 1024, 2048, 2),
                                          (256, 4096, 1024, 1), (130, 1024, 768, 1),
                                          (64, 1024, 2048, 4), (256, 1024, 3072, 8),
                                          (200, 2048, 1024, 2), (96, 1024, 512, 4),
                                          (256, 4096, 2048, 4), (256, 4096, 2048, 8)])
def test_lds_dma_decode_gemm(ring, bn, epi, M, N, K, splitk):
    """gdgemm.hip (global_load_lds ring) with each epilogue vs fp32 references: shallow
    (2 blocks/CU) and deep (1 block/CU) rings, split-K reduced by the separate pass or
    combined in-launch by the last-arriving slice (also for the SwiGLU epilogue); 128-row
    tiles and 256-row tiles (8 waves, 512 threads, row tails at M = 130 / 200 / 1 / 37), the
    latter also with the 6-slot ring of 32-deep k-steps (rows256deep: ns = 6)."""
    inl = ring.endswith("inlaunch")
    bm = 256 if ring.startswith("rows256") else 128 if ring.startswith("rows128") else 64
    if inl and splitk == 1:
        pytest.skip("in-launch combine needs split-K")
    if not ops.dgemm_supported(M, N, K, splitk, 1, epi, bn=bn, inlaunch=inl, bm=bm):
        pytest.skip("unsupported combination")
    kw = dict(ns=8 if ring.startswith("deep") else 6 if "deep" in ring else 0, inlaunch=inl,
              bm=bm)
    torch.manual_seed(M + N + K + epi + bn)
    eps = 1e-6
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    ssi = torch.rand(M, device=DEV) * K + 1.0
    y = (x.float() @ w.float().t()) * torch.rsqrt(ssi / K + eps)[:, None]
    if epi == ops.EPI_STORE:
        out = ops.dgemm(x, w, splitk=splitk, bn=bn, ss_in=ssi, eps=eps, **kw)
        _close(out, y, atol=2e-2 * y.abs().max().item())
        if inl:  # tickets re-armed by the last arriver: a second launch reuses them
            out2 = ops.dgemm(x, w, splitk=splitk, bn=bn, ss_in=ssi, eps=eps, **kw)
            assert torch.equal(out, out2)
    elif epi == ops.EPI_RESNORM:
        res = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
        res0 = res.clone()
        ln = torch.rand(N, device=DEV, dtype=torch.bfloat16) + 0.5
        ss = torch.zeros(M, device=DEV)
        a = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops.dgemm(x, w, splitk=splitk, bn=bn, out=res, epi=epi, ss_out=ss, a_out=a, ln_out=ln,
                  ss_in=ssi, eps=eps, **kw)
        want = y.to(torch.bfloat16).float() + res0.float()
        _close(res, want, atol=2e-2 * want.abs().max().item())
        _close(a, res.float() * ln.float(), atol=1e-2 * a.float().abs().max().item())
        assert torch.allclose(ss, res.float().pow(2).sum(-1), rtol=1e-3, atol=1e-2)
    else:
        out = ops.dgemm(x, w, splitk=splitk, bn=bn, epi=epi, ss_in=ssi, eps=eps, **kw)
        want = ref.silu_and_mul(y.to(torch.bfloat16)).float()
        _close(out, want, atol=2e-2 * want.abs().max().item())


@pytest.mark.parametrize("pf", [1, 2, 4, 8])
@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("scaled", [False, True])
@pytest.mark.parametrize("M,N,K,splitk", [(256, 1024, 3072, 4), (256, 1024, 2048, 2),
                                          (37, 1024, 3072, 8), (130, 2048, 1024, 2),
                                          (1, 256, 4096, 4), (256, 6144, 4096, 8)])
def test_register_ring_inlaunch_combine(pf, epi, scaled, M, N, K, splitk):
    """dgemm.hip SPL 2 (register-ring kernel, bn = 0): the K slices stored as sc1 slabs and
    combined by the tile's last-arriving slice inside the launch -- no reduce kernel -- with
    each epilogue (store, residual + next norm, SwiGLU), with and without the ss_in row
    scale, vs fp32 references; a second launch reuses the re-armed tickets bit-exactly."""
    if not ops.dgemm_supported(M, N, K, splitk, pf, epi, inlaunch=True):
        pytest.skip("unsupported combination")
    torch.manual_seed(M + N + K + epi + pf)
    eps = 1e-6
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    ssi = torch.rand(M, device=DEV) * K + 1.0 if scaled else None
    y = x.float() @ w.float().t()
    if scaled:
        y = y * torch.rsqrt(ssi / K + eps)[:, None]
    kw = dict(splitk=splitk, pf=pf, inlaunch=True, ss_in=ssi, eps=eps)
    if epi == ops.EPI_STORE:
        out = ops.dgemm(x, w, **kw)
        _close(out, y, atol=2e-2 * y.abs().max().item())
        out2 = ops.dgemm(x, w, **kw)
        assert torch.equal(out, out2)
    elif epi == ops.EPI_RESNORM:
        res = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
        res0 = res.clone()
        ln = torch.rand(N, device=DEV, dtype=torch.bfloat16) + 0.5
        ss = torch.zeros(M, device=DEV)
        a = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops.dgemm(x, w, out=res, epi=epi, ss_out=ss, a_out=a, ln_out=ln, **kw)
        want = y.to(torch.bfloat16).float() + res0.float()
        _close(res, want, atol=2e-2 * want.abs().max().item())
        _close(a, res.float() * ln.float(), atol=1e-2 * a.float().abs().max().item())
        assert torch.allclose(ss, res.float().pow(2).sum(-1), rtol=1e-3, atol=1e-2)
    else:
        out = ops.dgemm(x, w, epi=epi, **kw)
        want = ref.silu_and_mul(y.to(torch.bfloat16)).float()
        _close(out, want, atol=2e-2 * want.abs().max().item())


@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("M,N,K,splitk", [(256, 1024, 1024, 1), (256, 1024, 2048, 4),
                                          (200, 2048, 1024, 3), (256, 4096, 4096, 16),
                                          (37, 512, 14336, 16), (256, 6144, 4096, 10),
                                          (300, 1024, 1024, 2), (1, 768, 640, 5)])
def test_pgemm_split_k_inlaunch(epi, M, N, K, splitk):
    """The 256 x 256 pgemm body with K split over workgroups and the slices combined in the
    launch by every slice (dgemm bn=256, pgemm_sk_kernel): each epilogue with the ss_in row
    scale vs fp32 references, uneven K splits (3, 5, 10), row tails, two row tiles, and a
    second launch that reuses the re-armed tile counters."""
    if not ops.dgemm_supported(M, N, K, splitk, 1, epi, bn=256, inlaunch=True, bm=256):
        pytest.skip("unsupported combination")
    kw = dict(splitk=splitk, bn=256, bm=256, inlaunch=True)
    torch.manual_seed(M + N + K + epi + splitk)
    eps = 1e-6
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    ssi = torch.rand(M, device=DEV) * K + 1.0
    y = (x.float() @ w.float().t()) * torch.rsqrt(ssi / K + eps)[:, None]
    if epi == ops.EPI_STORE:
        out = ops.dgemm(x, w, ss_in=ssi, eps=eps, **kw)
        _close(out, y, atol=2e-2 * y.abs().max().item())
        out2 = ops.dgemm(x, w, ss_in=ssi, eps=eps, **kw)
        assert torch.equal(out, out2)
    elif epi == ops.EPI_RESNORM:
        res = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
        res0 = res.clone()
        ln = torch.rand(N, device=DEV, dtype=torch.bfloat16) + 0.5
        ss = torch.zeros(M, device=DEV)
        a = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops.dgemm(x, w, out=res, epi=epi, ss_out=ss, a_out=a, ln_out=ln, ss_in=ssi, eps=eps,
                  **kw)
        want = y.to(torch.bfloat16).float() + res0.float()
        _close(res, want, atol=2e-2 * want.abs().max().item())
        _close(a, res.float() * ln.float(), atol=1e-2 * a.float().abs().max().item())
        assert torch.allclose(ss, res.float().pow(2).sum(-1), rtol=1e-3, atol=1e-2)
    else:
        out = ops.dgemm(x, w, epi=epi, ss_in=ssi, eps=eps, **kw)
        want = ref.silu_and_mul(y.to(torch.bfloat16)).float()
        _close(out, want, atol=2e-2 * want.abs().max().item())
    # no combine timed out
    assert int(ops.gemm_counters(torch.device(DEV))[ops.GEMM_CTR_ERR].item()) == 0


@pytest.mark.parametrize("M", [1, 16, 37, 64, 100, 128, 200, 256, 300])
@pytest.mark.parametrize("N,K", [(1000, 64), (4100, 1024), (2056, 2048)])
def test_wide_row_gemm(M, N, K):
    """wgemm.hip (the decode LM head kernel): every row tile width (64/128/256 rows per
    workgroup, and > 256 rows over several), partial column tiles (N % 8 != 0 included)
    vs an fp32 matmul."""
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    # output rows padded to a multiple of 8 (16-byte aligned row starts); N itself need not be
    out = torch.full((M, N + (-N) % 8), float("nan"), device=DEV, dtype=torch.bfloat16)[:, :N]
    ops.wgemm(x, w, out=out)
    exp = x.float() @ w.float().T
    _close(out, exp, atol=0.02 * math.sqrt(K / 64), rtol=1e-2)


def test_wide_row_gemm_strided_rows_in_graph():
    """Strided input rows (a view of a larger buffer) and replay from a captured graph."""
    torch.manual_seed(1)
    buf = torch.randn(256, 1024 + 64, device=DEV, dtype=torch.bfloat16)
    x = buf[:, :1024]
    w = torch.randn(3000, 1024, device=DEV, dtype=torch.bfloat16) * 0.05
    out = torch.empty(256, 3000, device=DEV, dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ops.wgemm(x, w, out=out)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        ops.wgemm(x, w, out=out)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    _close(out, x.float() @ w.float().T, atol=0.1, rtol=1e-2)


@pytest.mark.parametrize("qk_norm", [True, False])
@pytest.mark.parametrize("fp8", [False, True])
def test_qk_norm_rope_cache_decode_mode(qk_norm, fp8):
    """decode=True (per-token V writes, one token per sequence) writes the same cache as the
    reference; a slot of -1 writes nothing."""
    torch.manual_seed(5)
    T, hq, hkv, D, BS, NB = 77, 16, 8, 128, 32, 40
    qkv = torch.randn(T, (hq + 2 * hkv) * D, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), dtype=torch.int64)
    slots = torch.randperm(NB * BS)[:T].to(torch.int64)
    slots[7] = -1
    cs = ref.rope_cos_sin(4096, D, 1e6)
    qw = torch.randn(D).bfloat16() if qk_norm else None
    kw = torch.randn(D).bfloat16() if qk_norm else None
    kc, vc = torch.zeros(NB, hkv, BS, D).bfloat16(), torch.zeros(NB, hkv, BS // 8, D, 8).bfloat16()
    q_ref = torch.empty(T, hq, D).bfloat16()
    ref.qk_norm_rope_cache(qkv, q_ref, kc, vc, pos, slots, cs, qw, kw, hq, hkv, 1e-6)
    dt = torch.float8_e4m3fn if fp8 else torch.bfloat16
    kg = torch.zeros(NB, hkv, BS, D, device=DEV, dtype=dt)
    vg = torch.zeros(NB, hkv, BS // 8, D, 8, device=DEV, dtype=dt)
    if fp8:
        kg, vg = kg.view(torch.uint8), vg.view(torch.uint8)
    q_out = torch.empty(T, hq, D, device=DEV, dtype=torch.bfloat16)
    ops.qk_norm_rope_cache(qkv.to(DEV), q_out, kg, vg, pos.to(DEV), slots.to(DEV), cs.to(DEV),
                           None if qw is None else qw.to(DEV), None if kw is None else kw.to(DEV),
                           hq, hkv, 1e-6, decode=True)
    _close(q_out, q_ref, atol=3e-2, rtol=2e-2)
    if fp8:
        _close(kg.view(torch.float8_e4m3fn).float(), kc.float().to(torch.float8_e4m3fn).float(),
               atol=0.1, rtol=0.13)
        _close(vg.view(torch.float8_e4m3fn).float(), vc.float().to(torch.float8_e4m3fn).float(),
               atol=0)
    else:
        _close(kg, kc, atol=3e-2, rtol=2e-2)
        _close(vg, vc, atol=0)


@pytest.mark.parametrize("km", [16, 32])
@pytest.mark.parametrize("epi", [0, 1])
@pytest.mark.parametrize("M,N,K", [(1, 1024, 2048), (37, 1024, 3072), (256, 1024, 2048),
                                   (200, 4096, 1024), (300, 96, 256)])
def test_kgemm_in_workgroup_splitk(km, epi, M, N, K):
    """kgemm.hip (K split over the workgroup's waves, partials summed in LDS) with the store
    and residual/next-norm epilogues and the ss_in row scale vs fp32 references; a second
    launch gives identical bits (no cross-workgroup state)."""
    torch.manual_seed(M + N + K + epi + km)
    eps = 1e-6
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    ssi = torch.rand(M, device=DEV) * K + 1.0
    y = (x.float() @ w.float().t()) * torch.rsqrt(ssi / K + eps)[:, None]
    if epi == 0:
        out = ops.dgemm(x, w, ss_in=ssi, eps=eps, km=km)
        _close(out, y, atol=2e-2 * y.abs().max().item())
        assert torch.equal(out, ops.dgemm(x, w, ss_in=ssi, eps=eps, km=km))
    else:
        res = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
        res0 = res.clone()
        ln = torch.rand(N, device=DEV, dtype=torch.bfloat16) + 0.5
        ss = torch.zeros(M, device=DEV)
        a = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops.dgemm(x, w, out=res, epi=epi, ss_out=ss, a_out=a, ln_out=ln, ss_in=ssi, eps=eps,
                  km=km)
        want = y.to(torch.bfloat16).float() + res0.float()
        _close(res, want, atol=2e-2 * want.abs().max().item())
        _close(a, res.float() * ln.float(), atol=1e-2 * a.float().abs().max().item())
        assert torch.allclose(ss, res.float().pow(2).sum(-1), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("num_parts,part_size", [(4, 8192), (32, 1024), (128, 256)])
def test_paged_attention_decode_long_context(num_parts, part_size):
    """Long-context decode (up to 32k cached tokens per sequence, Llama-3-70B's 64/8 heads
    per rank shape): unsplit, and split-KV with the partition combine (the engine's adaptive
    split picks partitions like these when few sequences carry long contexts)."""
    lens = [32768, 20001, 9000, 4097, 1]
    seqs = [(kv, 1) for kv in lens]
    hq, hkv = 64, 8
    q, kc, vc, bt, sl, qs = _setup_attn(seqs, hq, hkv, 32, seed=num_parts)
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q, kc, vc, bt, sl, qs, scale)
    out = torch.empty_like(q).to(DEV)
    ws = ops.decode_workspace(len(seqs), hkv, hq // hkv, num_parts, DEV)
    ops.paged_attention_decode(out, q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), sl.to(DEV),
                               hq // hkv, scale, workspace=ws, num_parts=num_parts,
                               part_size=part_size)
    _close(out, exp, atol=2e-2, rtol=2e-2)


def test_paged_attention_decode_rejects_oversized_partition():
    """A partition longer than ops.DECODE_MAX_PART is refused on the host (the kernel keeps
    one cache block id per 128-token wave step in a VGPR lane: 64 steps)."""
    q, kc, vc, bt, sl, qs = _setup_attn([(100, 1), (7, 1)], 16, 8, 32, seed=3)
    out = torch.empty_like(q).to(DEV)
    ws = ops.decode_workspace(2, 8, 2, 1, DEV)
    with pytest.raises(RuntimeError, match="part_size"):
        ops.paged_attention_decode(out, q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV),
                                   sl.to(DEV), 2, 0.1, workspace=ws, num_parts=1,
                                   part_size=2 * ops.DECODE_MAX_PART)


@pytest.mark.parametrize("num_parts,part_size", [(4, 8192), (64, 512), (128, 256), (32, 1024)])
def test_paged_attention_decode_fused_long_context(num_parts, part_size):
    """The engine's decode kernel (fused prologue) at long context with split-KV partitions."""
    test_paged_attention_decode_fused(16, 8, True, num_parts, part_size,
                                      lens=[8001, 1, 20001, 32768, 4095])


@pytest.mark.parametrize("num_parts,part_size", [(32, 256), (64, 256)])
def test_paged_attention_decode_fused_engine_split_plans(num_parts, part_size):
    """The split-KV plans the engine picks for one 8k-16k sequence (qwen3-0.6b shapes)."""
    test_paged_attention_decode_fused(16, 8, True, num_parts, part_size,
                                      lens=[8001, 6501, 8192, 1, 7000])


def test_paged_attention_prefill_deep_context():
    """Chunked prefill deep into a long prompt: 512-token chunks whose causal window reaches
    back over 16k cached tokens (plus a short fresh prompt in the same launch)."""
    seqs = [(16384, 512), (12000, 300), (700, 700)]
    hq, hkv = 16, 8
    q, kc, vc, bt, sl, qs = _setup_attn(seqs, hq, hkv, 32, seed=3)
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q, kc, vc, bt, sl, qs, scale)
    ts, tr = _tiles(seqs, hq // hkv, 128)
    out = torch.empty_like(q).to(DEV)
    ops.paged_attention_prefill(out, q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), sl.to(DEV),
                                qs.to(DEV), ts.to(DEV), tr.to(DEV), hq // hkv, scale,
                                tile_rows=128)
    _close(out, exp, atol=2e-2, rtol=2e-2)


def _v_tokens(vc, bt, s, n, bs=32):
    """[n, Hkv, D] V rows of sequence s's first n tokens from a [NB, Hkv, BS/8, D, 8] cache."""
    rows = []
    for p in range(n):
        b = int(bt[s, p // bs])
        rows.append(vc[b, :, (p % bs) // 8, :, p % 8])
    return torch.stack(rows)


@pytest.mark.parametrize("num_parts,part_size", [(1, 4096), (3, 512)])
def test_v_tail_decode_matches_the_plain_cache_path(num_parts, part_size):
    """V tail (AttnParams.v_tail): decode steps write the new token's V to its sequence's
    tail and whole 8-token groups to the cache; readers take the partial group from the tail.
    Against a twin cache on the plain per-token path, over 20 steps (fused steps, plus mixed
    steps through the writer kernel + the plain decode kernel): bit-identical attention
    outputs, and identical V for every completed group."""
    hq, hkv, D, BS = 16, 8, 128, 32
    lens = [1, 5, 8, 13, 31, 200, 777]
    steps = 20
    seqs = [(kv + steps, 1) for kv in lens]  # blocks for the prompt + every decode token
    _, kc, vc, bt, _, _ = _setup_attn(seqs, hq, hkv, BS, seed=7)
    B, G = len(lens), hq // hkv
    g = torch.Generator().manual_seed(3)
    cs = ref.rope_cos_sin(4096, D, 1e6).to(DEV)
    qw = torch.randn(D, generator=g).bfloat16().to(DEV)
    kw = torch.randn(D, generator=g).bfloat16().to(DEV)
    btg = bt.to(DEV)
    kA, vA = kc.to(DEV), vc.to(DEV)
    kB, vB = kA.clone(), vA.clone()
    tail = torch.zeros(B, hkv, 8, D, dtype=torch.bfloat16, device=DEV)
    tslot = torch.arange(B, dtype=torch.int32, device=DEV)
    for s, n in enumerate(lens):  # the prompt's partial group -> tail (like fill_tail)
        g0 = n & ~7
        for p in range(g0, n):
            b = int(bt[s, p // BS])
            tail[s, :, p - g0] = vB[b, :, (p % BS) // 8, :, p % 8]
    scale = 1 / math.sqrt(D)
    cur = list(lens)
    for step in range(steps):
        pos = torch.tensor(cur, dtype=torch.int64)
        slots = torch.tensor([int(bt[s, cur[s] // BS]) * BS + cur[s] % BS for s in range(B)],
                             dtype=torch.int64).to(DEV)
        sl = torch.tensor([c + 1 for c in cur], dtype=torch.int32, device=DEV)
        qkv = torch.randn(B, (hq + 2 * hkv) * D, generator=g).bfloat16().to(DEV)
        outs = []
        for kcache, vcache, vt in ((kA, vA, None), (kB, vB, tail)):
            out = torch.empty(B, hq, D, dtype=torch.bfloat16, device=DEV)
            ws = ops.decode_workspace(B, hkv, G, num_parts, DEV)
            if step % 5 == 4:  # a mixed step: writer kernel (span role) + plain decode kernel
                q = torch.empty(B, hq, D, dtype=torch.bfloat16, device=DEV)
                ops.qk_norm_rope_cache(qkv, q, kcache, vcache, pos.to(DEV), slots, cs, qw, kw,
                                       hq, hkv, 1e-6, True, decode=False, v_tail=vt,
                                       tail_slot=tslot, num_decode=B)
                ops.paged_attention_decode(out, q, kcache, vcache, btg, sl, G, scale,
                                           workspace=ws, num_parts=num_parts,
                                           part_size=part_size, v_tail=vt, tail_slot=tslot)
            else:
                ops.paged_attention_decode_fused(out, qkv, kcache, vcache, btg, sl, pos.to(DEV),
                                                 slots, cs, qw, kw, G, scale, 1e-6, workspace=ws,
                                                 num_parts=num_parts, part_size=part_size,
                                                 v_tail=vt, tail_slot=tslot)
            outs.append(out)
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1]), (step, (outs[0].float() - outs[1].float()).abs().max())
        cur = [c + 1 for c in cur]
    vA_, vB_ = vA.cpu(), vB.cpu()
    for s, n in enumerate(cur):
        full = n & ~7
        assert torch.equal(_v_tokens(vA_, bt, s, full), _v_tokens(vB_, bt, s, full)), s
    assert torch.equal(kA, kB)


# ----------------------------------------------------------------------------- prefill GEMM
@pytest.mark.parametrize("M,N,K", [(1, 256, 64), (300, 512, 128), (256, 1024, 1024),
                                   (1000, 768, 2048), (4096, 4096, 1024), (517, 256, 4096)])
def test_pgemm_matches_fp32(M, N, K):
    """pgemm (256x256 tiles, phased LDS-DMA pipeline) vs an fp32 reference, asymmetric random
    operands, M not a multiple of the tile, K from one to 64 K tiles."""
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * 0.05).bfloat16()
    y = ops.pgemm(x.to(DEV), w.to(DEV))
    exp = x.float() @ w.float().t()
    err = (y.float().cpu() - exp).abs().max().item()
    assert err <= 2e-2 * exp.abs().max().item() + 1e-2, err


def test_pgemm_identity_and_layout():
    """A = I on the first K columns, W asymmetric: catches a transposed C write or a wrong
    fragment map exactly (cdna_hip_programming.md section 3)."""
    M, N, K = 256, 512, 256
    x = torch.zeros(M, K)
    x[:, :].fill_diagonal_(1.0)
    w = (torch.arange(N * K, dtype=torch.float32).reshape(N, K) % 61 - 30) / 8
    y = ops.pgemm(x.bfloat16().to(DEV), w.bfloat16().to(DEV)).float().cpu()
    assert torch.equal(y, (x @ w.bfloat16().float().t()).bfloat16().float())


@pytest.mark.parametrize("M,F,K", [(300, 256, 256), (2048, 1536, 1024)])
def test_pgemm_silu_epilogue(M, F, K):
    g = torch.Generator().manual_seed(F + K)
    x = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(2 * F, K, generator=g) * 0.05).bfloat16()
    y = ops.pgemm(x.to(DEV), w.to(DEV), silu=True).float().cpu()
    exp = ref.pgemm(x, w, silu=True).float()
    assert (y - exp).abs().max().item() <= 3e-2 * exp.abs().max().item() + 1e-2


@pytest.mark.parametrize("counts", [[300, 0, 517, 1, 256, 0, 0, 40], [0, 0, 1024], [5]])
def test_pgemm_grouped(counts):
    """Expert-grouped form over device-side offsets: empty groups, 1-row groups and groups that
    are not a multiple of the tile; every group's rows use its own weight."""
    G = len(counts)
    M = sum(counts)
    N, K = 512, 256
    g = torch.Generator().manual_seed(G + M)
    x = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(G, N, K, generator=g) * 0.05).bfloat16()
    offs = torch.tensor(counts).cumsum(0).int()
    for silu in (False, True):
        y = ops.pgemm(x.to(DEV), w.to(DEV), silu=silu, offs=offs.to(DEV)).float().cpu()
        exp = ref.pgemm(x, w, silu, offs).float()
        assert (y - exp).abs().max().item() <= 3e-2 * exp.abs().max().item() + 1e-2, silu


def test_h2d_stage_kernel_copies_pinned_host_memory():
    """The in-stream staging copy (a kernel reading the pinned buffer's device mapping)."""
    for n in (1, 15, 16, 4099, 65536 + 7):
        src = torch.randint(0, 255, (n,), dtype=torch.uint8).pin_memory()
        dst = torch.zeros(n, dtype=torch.uint8, device=DEV)
        torch.ops.akap.h2d_stage(dst, src)
        torch.cuda.synchronize()
        assert torch.equal(dst.cpu(), src)
