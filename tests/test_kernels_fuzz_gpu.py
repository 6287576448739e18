"""Hypothesis shape fuzzing of the HIP kernels against their fp32 torch references
("hypothesis shape fuzzing").  Small example counts: every example is a real
kernel launch on the MI355X."""
import math

import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from aws_k8s_ansible_provisioner_amd import ops
from aws_k8s_ansible_provisioner_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
FUZZ = settings(max_examples=12, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])


def _close(a, b, atol, rtol=0.0):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    assert bool((err <= atol + rtol * b.abs()).all()), f"max err {err.max().item():.4g}"


@FUZZ
@given(st.integers(1, 300), st.sampled_from([8, 64, 1000, 1024, 2048, 4096, 5120, 8192]),
       st.booleans(), st.integers(0, 1000))
def test_fuzz_rmsnorm(rows, d, add, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(rows, d, generator=g).bfloat16()
    w = torch.randn(d, generator=g).bfloat16()
    if add:
        r = torch.randn(rows, d, generator=g).bfloat16()
        rg = r.to(DEV)
        out, _ = ops.fused_add_rms_norm(x.to(DEV), rg, w.to(DEV), 1e-6)
        s = (x.float() + r.float()).bfloat16()
        _close(rg, s, atol=0)
        _close(out, ref.rms_norm(s, w, 1e-6), atol=2e-2, rtol=2e-2)
    else:
        _close(ops.rms_norm(x.to(DEV), w.to(DEV), 1e-6), ref.rms_norm(x, w, 1e-6), atol=2e-2,
               rtol=2e-2)


@FUZZ
@given(st.integers(1, 200), st.sampled_from([8, 64, 768, 3072, 14336]), st.integers(0, 1000))
def test_fuzz_silu_and_mul(T, F, seed):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(T, 2 * F, generator=g) * 3).bfloat16()
    _close(ops.silu_and_mul(x.to(DEV)), ref.silu_and_mul(x), atol=3e-2, rtol=2e-2)


def _cache(lens, hkv, bs, g):
    D = 128
    nb = [math.ceil(L / bs) for L in lens]
    NB = sum(nb) + 2
    kc = torch.randn(NB, hkv, bs, D, generator=g).bfloat16()
    vc = torch.randn(NB, hkv, bs // 8, D, 8, generator=g).bfloat16()
    perm = torch.randperm(NB, generator=g)
    bt = torch.zeros(len(lens), max(nb), dtype=torch.int32)
    i = 0
    for s, n in enumerate(nb):
        bt[s, :n] = perm[i:i + n].to(torch.int32)
        i += n
    return kc, vc, bt


@FUZZ
@given(st.lists(st.integers(1, 1200), min_size=1, max_size=6),
       st.sampled_from([(16, 8), (32, 8), (64, 8), (8, 8), (28, 4)]),
       st.sampled_from([(1, 4096), (2, 640), (4, 384)]), st.integers(0, 1000))
def test_fuzz_decode_attention(lens, heads, split, seed):
    hq, hkv = heads
    parts, psize = split
    lens = [min(L, parts * psize) for L in lens]
    g = torch.Generator().manual_seed(seed)
    kc, vc, bt = _cache(lens, hkv, 32, g)
    B, G = len(lens), hq // hkv
    q = torch.randn(B, hq, 128, generator=g).bfloat16()
    sl = torch.tensor(lens, dtype=torch.int32)
    qs = torch.arange(B + 1, dtype=torch.int32)
    exp = ref.paged_attention(q, kc, vc, bt, sl, qs, 128 ** -0.5)
    out = torch.empty(B, hq, 128, dtype=torch.bfloat16, device=DEV)
    ws = ops.decode_workspace(B, hkv, G, parts, DEV)
    ops.paged_attention_decode(out, q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), sl.to(DEV), G,
                               128 ** -0.5, workspace=ws, num_parts=parts, part_size=psize)
    _close(out, exp, atol=3e-2, rtol=3e-2)


@FUZZ
@given(st.lists(st.tuples(st.integers(1, 700), st.integers(1, 300)), min_size=1, max_size=4),
       st.sampled_from([(16, 8), (32, 8), (8, 8)]), st.sampled_from([128, 256]),
       st.integers(0, 1000))
def test_fuzz_prefill_attention(seqs, heads, rows, seed):
    hq, hkv = heads
    seqs = [(max(kv, ql), ql) for kv, ql in seqs]  # new tokens <= context
    g = torch.Generator().manual_seed(seed)
    kc, vc, bt = _cache([kv for kv, _ in seqs], hkv, 32, g)
    G = hq // hkv
    qs = torch.zeros(len(seqs) + 1, dtype=torch.int32)
    for s, (_, ql) in enumerate(seqs):
        qs[s + 1] = qs[s] + ql
    q = torch.randn(int(qs[-1]), hq, 128, generator=g).bfloat16()
    sl = torch.tensor([kv for kv, _ in seqs], dtype=torch.int32)
    ts, tr = [], []
    for s, (_, ql) in enumerate(seqs):
        for r in range(0, ql * G, rows):
            ts.append(s)
            tr.append(r)
    exp = ref.paged_attention(q, kc, vc, bt, sl, qs, 128 ** -0.5)
    out = torch.empty_like(q).to(DEV)
    ops.paged_attention_prefill(out, q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), sl.to(DEV),
                                qs.to(DEV), torch.tensor(ts, dtype=torch.int32, device=DEV),
                                torch.tensor(tr, dtype=torch.int32, device=DEV), G, 128 ** -0.5,
                                tile_rows=rows)
    _close(out, exp, atol=3e-2, rtol=3e-2)


@FUZZ
@given(st.integers(1, 64), st.sampled_from([1000, 32000, 128256, 151936]), st.integers(0, 1000))
def test_fuzz_greedy_sampling(B, V, seed):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(B, V, generator=g).bfloat16().to(DEV)
    z = torch.zeros(B, device=DEV)
    tok, _ = ops.sample(logits, z, torch.zeros(B, dtype=torch.int32, device=DEV),
                        torch.ones(B, device=DEV), torch.arange(B, device=DEV),
                        torch.zeros(B, dtype=torch.int32, device=DEV))
    assert torch.equal(tok, logits.float().argmax(-1))


@FUZZ
@given(st.integers(1, 4096), st.sampled_from([(256, 1024), (1000, 64), (4096, 8)]),
       st.integers(0, 1000))
def test_fuzz_embedding(T, shape, seed):
    V, d = shape
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, V, (T,), generator=g)
    table = torch.randn(V, d, generator=g).bfloat16()
    _close(ops.embedding(ids.to(DEV), table.to(DEV)), ref.embedding(ids, table, 0, V), atol=0)


@FUZZ
@given(st.lists(st.tuples(st.integers(0, 40), st.integers(1, 150)), min_size=1, max_size=5),
       st.booleans(), st.booleans(), st.integers(0, 1000))
def test_fuzz_qk_norm_rope_cache(runs, qk_norm, fp8, seed):
    """Batches made of runs of consecutive slots at arbitrary offsets (prefill chunks,
    chunk edges, decode tokens, padding -1): every 8-token V group is either complete,
    partial or split across the kernel's 64-token spans."""
    hq, hkv, D, BS = 16, 8, 128, 32
    g = torch.Generator().manual_seed(seed)
    slots, base = [], 0
    for start, n in runs:
        if start == 0 and slots:
            slots.append(-1)
        base = (base + BS * 2 + start)  # disjoint slot ranges per run
        slots += list(range(base, base + n))
        base += n
    T = len(slots)
    NB = base // BS + 2
    slots = torch.tensor(slots, dtype=torch.int64)
    qkv = torch.randn(T, (hq + 2 * hkv) * D, generator=g).bfloat16()
    pos = torch.randint(0, 4000, (T,), generator=g)
    cs = ref.rope_cos_sin(4096, D, 1e6)
    qw = torch.randn(D, generator=g).bfloat16() if qk_norm else None
    kw = torch.randn(D, generator=g).bfloat16() if qk_norm else None
    dt = torch.uint8 if fp8 else torch.bfloat16
    kc = torch.zeros(NB, hkv, BS, D, dtype=dt)
    vc = torch.zeros(NB, hkv, BS // 8, D, 8, dtype=dt)
    q_ref = torch.empty(T, hq, D).bfloat16()
    kg, vg = kc.to(DEV), vc.to(DEV)
    ref.qk_norm_rope_cache(qkv, q_ref, kc, vc, pos, slots, cs, qw, kw, hq, hkv, 1e-6)
    q_out = torch.empty(T, hq, D, device=DEV, dtype=torch.bfloat16)
    ops.qk_norm_rope_cache(qkv.to(DEV), q_out, kg, vg, pos.to(DEV), slots.to(DEV), cs.to(DEV),
                           None if qw is None else qw.to(DEV), None if kw is None else kw.to(DEV),
                           hq, hkv, 1e-6)
    _close(q_out, q_ref, atol=3e-2, rtol=2e-2)
    if fp8:
        _close(ref.from_cache(kg.cpu()), ref.from_cache(kc), atol=1e-2, rtol=0.13)
        assert torch.equal(vg.cpu(), vc)
    else:
        _close(kg, kc, atol=3e-2, rtol=2e-2)
        assert torch.equal(vg.cpu(), vc)
