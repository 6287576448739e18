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
       st.sampled_from([(16, 8), (32, 8), (8, 8)]), st.sampled_from([64, 128]),
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
