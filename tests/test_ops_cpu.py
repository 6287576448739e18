"""CPU checks of the op references (the semantics every HIP kernel is tested against)
and of the Python-side glue around them.  The GPU kernels are compared against these
same references in tests/test_kernels_gpu.py."""
import math

import pytest
import torch

from aws_k8s_ansible_provisioner_amd import ops
from aws_k8s_ansible_provisioner_amd.ops import reference as ref


def _moe_dense(h, w13, w2, w, ids):
    """Dense fp32 formulation: every token through every expert, masked by routing."""
    T, d = h.shape
    E = w13.shape[0]
    F = w13.shape[1] // 2
    out = torch.zeros(T, d)
    for e in range(E):
        y = h.float() @ w13[e].float().t()
        a = torch.nn.functional.silu(y[:, :F]) * y[:, F:]
        y2 = a @ w2[e].float().t()
        gate = ((ids == e).float() * w).sum(-1, keepdim=True)
        out += gate * y2
    return out


def test_fused_moe_reference_matches_dense():
    torch.manual_seed(0)
    T, E, K, d, F = 9, 4, 2, 32, 24
    h = torch.randn(T, d, dtype=torch.bfloat16)
    w13 = (torch.randn(E, 2 * F, d) * 0.2).bfloat16()
    w2 = (torch.randn(E, d, F) * 0.2).bfloat16()
    w, ids = ref.moe_topk_softmax(torch.randn(T, E), K)
    got = ops.fused_moe(h, w13, w2, w, ids).float()
    exp = _moe_dense(h, w13, w2, w, ids)
    assert torch.allclose(got, exp, atol=3e-2, rtol=3e-2)


def test_moe_align_reference_layout():
    ids = torch.tensor([[0, 2], [2, 1], [0, 2]], dtype=torch.int32)
    s, off, npad = ops.moe_align(ids, 4, 4)
    assert off.tolist() == [0, 4, 8, 12, 12]
    assert int(npad) == 12
    flat = ids.reshape(-1)
    for e in range(4):
        seg = s[off[e]:off[e + 1]]
        real = seg[seg < flat.numel()]
        assert sorted(real.tolist()) == (flat == e).nonzero().flatten().tolist()


def test_moe_expert_rows_skip_empty_slots():
    """EP fixed-dispatch receive buffers at prefill sizes: rows with local expert id -1 (empty
    slots) sort into a dummy group past the last offset and are never computed; every real
    row matches its expert's SwiGLU FFN."""
    from aws_k8s_ansible_provisioner_amd.models.config import get_config
    from aws_k8s_ansible_provisioner_amd.models.moe import MoEBlock
    from aws_k8s_ansible_provisioner_amd.parallel.state import ParallelState

    cfg = get_config("tiny-mixtral8")
    blk = MoEBlock(cfg, ParallelState(rank=0, world_size=1, tp_size=1), "cpu", torch.bfloat16,
                   torch.Generator().manual_seed(0), full_then_shard=False, mode="tp")
    torch.manual_seed(5)
    R = 96
    x = torch.randn(R, cfg.hidden_size, dtype=torch.bfloat16)
    e = torch.randint(0, blk.e_local, (R,))
    e[torch.rand(R) < 0.4] = -1
    y = blk._expert_rows(x, e.to(torch.int32))
    real = e >= 0
    one = torch.ones(R, 1)
    exp = ops.fused_moe(x[real], blk.w13, blk.w2, one[real], e[real].view(-1, 1).to(torch.int32))
    assert torch.allclose(y[real].float(), exp.float(), atol=3e-2, rtol=3e-2)


def test_moe_capacity_covers_worst_case():
    for n, E, b in [(1, 8, 64), (512, 8, 64), (7, 64, 16)]:
        cap = ops.moe_capacity(n, E, b)
        assert cap % b == 0 and cap >= n + E * (b - 1)


def test_paged_attention_reference_vs_dense_causal():
    torch.manual_seed(1)
    Hq, Hkv, D, BS = 4, 2, 64, 32
    lens = [5, 53]
    nb = 8
    kc = torch.zeros(nb, Hkv, BS, D)
    vc = torch.zeros(nb, Hkv, BS // 8, D, 8)
    tables = torch.tensor([[3, 5, 0, 0], [1, 6, 0, 0]], dtype=torch.int32)
    ks, vs = [], []
    for b, L in enumerate(lens):
        k = torch.randn(L, Hkv, D)
        v = torch.randn(L, Hkv, D)
        slots = torch.tensor([int(tables[b, t // BS]) * BS + t % BS for t in range(L)])
        ref.write_cache(k, v, kc, vc, slots)
        ks.append(k)
        vs.append(v)
    q = torch.randn(sum(lens), Hq, D)
    q_start = torch.tensor([0, lens[0], sum(lens)], dtype=torch.int32)
    out = ref.paged_attention(q, kc, vc, tables, torch.tensor(lens), q_start, D ** -0.5)
    G = Hq // Hkv
    for b, L in enumerate(lens):
        qb = q[q_start[b]:q_start[b + 1]]
        K = ks[b].repeat_interleave(G, 1)
        V = vs[b].repeat_interleave(G, 1)
        s = torch.einsum("qhd,khd->hqk", qb, K) * D ** -0.5
        s = s.masked_fill(torch.ones(L, L).triu(1).bool()[None], -math.inf)
        o = torch.einsum("hqk,khd->qhd", s.softmax(-1), V)
        assert torch.allclose(out[q_start[b]:q_start[b + 1]], o, atol=1e-5)


def test_v_cache_group_layout_roundtrip():
    BS, D, Hkv = 32, 32, 2
    kc = torch.zeros(4, Hkv, BS, D)
    vc = torch.zeros(4, Hkv, BS // 8, D, 8)
    k = torch.randn(40, Hkv, D)
    v = torch.randn(40, Hkv, D)
    slots = torch.arange(40) + 32
    ref.write_cache(k, v, kc, vc, slots)
    K, V = ref.gather_kv(kc, vc, torch.tensor([1, 2], dtype=torch.int32), 40)
    assert torch.equal(K, k) and torch.equal(V, v)
    # token o of block b sits at v_cache[b, h, o // 8, :, o % 8]
    assert torch.equal(vc[1, 0, 1, :, 3], v[11, 0])


def test_k_cache_fragment_layout():
    """K is stored [chunk][tile tt][k-step][row r][32 dims] per 32-token chunk, with chunk
    token o = 8*(r>>2) + 4*tt + (r&3) (the decode kernel's MFMA operand order)."""
    BS, D, H = 64, 128, 2
    kc = torch.zeros(3, H, BS, D)
    vals = torch.randn(BS, H, D)
    for o in range(BS):
        ref.write_k(kc, 1, o, vals[o])
    flat = kc[1].reshape(H, -1)
    for o in [0, 3, 4, 5, 9, 31, 32, 45, 63]:
        c, oo = divmod(o, 32)
        tt, r = (oo >> 2) & 1, ((oo >> 3) << 2) | (oo & 3)
        for d in [0, 31, 32, 100, 127]:
            off = c * 32 * 128 + tt * 2048 + (d // 32) * 512 + r * 32 + d % 32
            assert flat[0, off] == vals[o, 0, d]
    assert torch.equal(ref.k_tokens(kc, torch.tensor([1])), vals)
    # the permutation is a bijection over each chunk
    assert sorted(ref.K_CHUNK_POS) == list(range(32))


def test_block_size_must_be_multiple_of_32():
    from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig
    with pytest.raises(ValueError):
        EngineConfig(block_size=16)
    EngineConfig(block_size=64)


def test_sampler_reference_topk_topp_support():
    torch.manual_seed(2)
    V = 50
    logits = torch.randn(64, V)
    temp = torch.full((64,), 0.8)
    top_k = torch.full((64,), 5, dtype=torch.int32)
    top_p = torch.full((64,), 1.0)
    toks, lps = ref.sample(logits, temp, top_k, top_p, torch.arange(64), torch.zeros(64))
    for i in range(64):
        assert int(toks[i]) in torch.topk(logits[i], 5).indices.tolist()
        assert float(lps[i]) <= 0.0
    greedy, _ = ref.sample(logits, torch.zeros(64), top_k, top_p, torch.arange(64),
                           torch.zeros(64))
    assert torch.equal(greedy, logits.argmax(-1))


def test_rope_llama3_scaling_keeps_high_freqs():
    plain = ref.rope_cos_sin(20000, 128, 500000.0)
    sc = ref.rope_cos_sin(20000, 128, 500000.0, {"rope_type": "llama3", "factor": 8.0,
                                              "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                              "original_max_position_embeddings": 8192})
    # highest frequencies (first dims) are unscaled, lowest are divided by the factor
    assert torch.allclose(plain[:, :4], sc[:, :4])
    assert not torch.allclose(plain[:, 124:128], sc[:, 124:128], atol=1e-3)


def test_gemm_splitk_fills_chip():
    for M, N, K in [(64, 1024, 4096), (256, 4096, 1024), (512, 151936, 1024)]:
        s = ops.gemm_splitk(M, N, K)
        tiles = ((M + 63) // 64) * ((N + 63) // 64)
        assert tiles * s >= 256 or K // (s * 2) < 256


def test_native_library_registers_all_ops():
    """_C.so must load on a CPU host too (op schemas are checked at registration: a C++/
    schema mismatch aborts the process at import on the GPU box)."""
    import os
    if not os.path.exists(ops._LIB):
        pytest.skip("extension not built")
    assert ops.load_native(), ops._load_error
    for name in ("rmsnorm", "fused_add_rmsnorm", "qk_norm_rope_cache", "paged_attention_prefill",
                 "paged_attention_decode", "paged_attention_decode_fused", "sample", "gemm",
                 "moe_gemm", "moe_combine", "car_all_reduce", "kv_gather", "embedding",
                 "embedding_prep", "wgemm", "argmax", "car_all_to_all", "car_all_gather",
                 "paged_attention_prefill_qprep"):
        assert hasattr(torch.ops.akap, name), name


def test_prefill_qprep_cpu_path_uses_the_written_q():
    """On the CPU the qprep argument is ignored: qk_norm_rope_cache (reference) writes every q
    row whatever q_rows says, and the reference attention reads q -- the same result as the
    two-pass call."""
    import math
    torch.manual_seed(0)
    hq, hkv, D, BS = 4, 2, 128, 32
    T = 20
    qkv = torch.randn(T, (hq + 2 * hkv) * D).bfloat16()
    kc = torch.zeros(2, hkv, BS, D, dtype=torch.bfloat16)
    vc = torch.zeros(2, hkv, BS // 8, D, 8, dtype=torch.bfloat16)
    pos = torch.arange(T, dtype=torch.int64)
    slots = torch.arange(T, dtype=torch.int64)
    cs = ops.reference.rope_cos_sin(64, D, 1e6)
    q = torch.empty(T, hq, D, dtype=torch.bfloat16)
    ops.qk_norm_rope_cache(qkv, q, kc, vc, pos, slots, cs, None, None, hq, hkv, 1e-6, True,
                           q_rows=3)
    bt = torch.tensor([[0, 1]], dtype=torch.int32)
    sl = torch.tensor([T], dtype=torch.int32)
    qs = torch.tensor([0, T], dtype=torch.int32)
    ts = torch.zeros(1, dtype=torch.int32)
    tr = torch.zeros(1, dtype=torch.int32)
    a = torch.empty_like(q)
    b = torch.empty_like(q)
    ops.paged_attention_prefill(a, q, kc, vc, bt, sl, qs, ts, tr, 2, 1 / math.sqrt(D))
    ops.paged_attention_prefill(b, q, kc, vc, bt, sl, qs, ts, tr, 2, 1 / math.sqrt(D),
                                qprep=(qkv, pos, cs, None, 1e-6))
    assert torch.equal(a, b)
    assert torch.isfinite(a.float()).all()


def test_embedding_prep_reference_semantics():
    """CPU path of ops.embedding_prep (the decode prologue): residual = embedding rows (zeros
    outside the vocab shard), a_out = residual * ln, ss = row sums of squares, zbuf zeroed."""
    g = torch.Generator().manual_seed(5)
    V, d, T = 50, 64, 7
    table = (torch.randn(V, d, generator=g) * 0.5).bfloat16()
    ln = (torch.rand(d, generator=g) + 0.5).bfloat16()
    ids = torch.tensor([0, 3, 49, 60, 7, 7, 20])
    res = torch.empty(T, d, dtype=torch.bfloat16)
    a = torch.empty_like(res)
    ss = torch.empty(T)
    z = torch.full((4, T), 3.0)
    ops.embedding_prep(ids, table, ln, res, a, ss, z, 0, 40)  # shard [0, 40)
    x = ref.embedding(ids, table[:40], 0, 40)
    assert torch.equal(res, x) and float(res[2].abs().sum()) == 0.0  # id 49: other shard
    assert torch.allclose(a.float(), (x.float() * ln.float()).bfloat16().float())
    assert torch.allclose(ss, x.float().pow(2).sum(-1), rtol=1e-5)
    assert float(z.abs().max()) == 0.0


def test_fp8_cache_roundtrip_reference():
    BS, D, H = 32, 128, 2
    kc = torch.zeros(3, H, BS, D, dtype=torch.uint8)
    vc = torch.zeros(3, H, BS // 8, D, 8, dtype=torch.uint8)
    k = torch.randn(40, H, D) * 3
    v = torch.randn(40, H, D) * 3
    k[0, 0, 0] = 1000.0  # saturates to 448
    slots = torch.arange(40) + 32
    ref.write_cache(k, v, kc, vc, slots)
    K, V = ref.gather_kv(kc, vc, torch.tensor([1, 2], dtype=torch.int32), 40)
    assert K.dtype == torch.bfloat16
    assert float(K[0, 0, 0]) == 448.0
    rel = ((K.float() - k).abs() / (k.abs() + 1e-2))[1:]
    assert float(rel.median()) < 0.07  # e4m3: 3 mantissa bits
    assert torch.equal(V.float(), v.float().to(torch.float8_e4m3fn).float())


def test_fused_decode_gemm_reference_semantics():
    """CPU path of ops.dgemm: prologue (plain / add+RMSNorm / SiLU*up) then GEMM."""
    import torch
    from aws_k8s_ansible_provisioner_amd import ops
    from aws_k8s_ansible_provisioner_amd.ops import reference as ref

    torch.manual_seed(0)
    M, N, K = 5, 48, 64
    w = torch.randn(N, K, dtype=torch.bfloat16)
    x = torch.randn(M, K, dtype=torch.bfloat16)
    r = torch.randn(M, K, dtype=torch.bfloat16)
    ln = torch.rand(K, dtype=torch.bfloat16) + 0.5
    rout = torch.empty_like(r)
    y = ops.dgemm(x, w, ops.PRO_ADDNORM, residual=r, residual_out=rout, ln=ln, eps=1e-6)
    s = (x.float() + r.float()).to(torch.bfloat16)
    assert torch.equal(rout, s)
    want = ref.rms_norm(s, ln, 1e-6).float() @ w.float().t()
    assert torch.allclose(y.float(), want, atol=0.1, rtol=0.02)
    g = torch.randn(M, 2 * K, dtype=torch.bfloat16)
    y2 = ops.dgemm(g, w, ops.PRO_SILU)
    want2 = ref.silu_and_mul(g).float() @ w.float().t()
    assert torch.allclose(y2.float(), want2, atol=0.1, rtol=0.02)
    assert torch.allclose(ops.dgemm(x, w).float(), x.float() @ w.float().t(), atol=0.1, rtol=0.02)


def test_fused_decode_gemm_support_rules():
    from aws_k8s_ansible_provisioner_amd import ops

    assert ops.dgemm_supported(256, 4096, 1024, 1, 2)
    assert ops.dgemm_supported(256, 1024, 2048, 4, 4)
    assert not ops.dgemm_supported(256, 1024, 2048, 4, 3)    # prefetch depth 1|2|4
    assert not ops.dgemm_supported(256, 1022, 1024, 1, 1)    # N % 4
    assert not ops.dgemm_supported(256, 1024, 1024, 8, 4)    # K/split not a multiple of 64*pf


def test_qprep_position_invariant_check():
    """the q-prep prefill kernel rotates by key index, not by `positions`; the
    debug check (AKAP_DEBUG_CHECKS=1) refuses batches where the two differ or where the
    rotary table is too short."""
    import pytest

    from aws_k8s_ansible_provisioner_amd import ops

    q_start = torch.tensor([0, 3, 5], dtype=torch.int32)
    seq_lens = torch.tensor([10, 2], dtype=torch.int32)
    pos = torch.tensor([7, 8, 9, 0, 1])
    ops.check_qprep_positions(pos, seq_lens, q_start, 16)
    with pytest.raises(ValueError, match="key indices"):
        ops.check_qprep_positions(torch.tensor([7, 8, 10, 0, 1]), seq_lens, q_start, 16)
    with pytest.raises(ValueError, match="rotary"):
        ops.check_qprep_positions(pos, seq_lens, q_start, 8)


def test_tuner_shape_class_pruning():
    """only the anchor batch sizes search every GEMM variant; the others
    time the top choices of their two neighbouring anchors."""
    from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner as gt

    ms = [16, 24, 32, 48, 64, 80, 96, 112, 128, 160, 192, 224, 256]
    a = gt.anchor_ms(ms)
    assert a == [16, 64, 128, 256]
    ranks = {16: [("x",), ("y",), ("z",), ("w",)], 64: [("y",), ("q",), ("torch",)],
             128: [("k",)], 256: [("g",)]}
    assert gt._neighbour_allowed(64, a, ranks.get) is None
    assert gt._neighbour_allowed(48, a, ranks.get) == {("x",), ("y",), ("z",), ("q",),
                                                       ("torch",)}
    assert gt._neighbour_allowed(200, a, ranks.get) == {("k",), ("g",)}
    assert gt.anchor_ms([16, 32, 64]) == [16, 32, 64]


def test_tuner_rotation_keeps_weights_cold():
    """Candidates are timed on enough layer copies to stream >= 768 MB per rotation (3x the
    MALL) and at least 4 -- not on every layer (Llama-3-8B cold tuning time)."""
    from aws_k8s_ansible_provisioner_amd.ops.gemm_tuner import _rot

    def layers(n, mb):
        return [torch.empty(int(mb * (1 << 20)) // 2, dtype=torch.bfloat16) for _ in range(n)]

    assert len(_rot(layers(28, 8.4))) == 28  # Qwen3 qkv: all 28 (235 MB in total)
    assert len(_rot(layers(32, 235))) == 4  # Llama-3-8B gate_up: 4 x 235 MB
    assert len(_rot(layers(32, 50))) == 16  # Llama-3-8B qkv
    assert len(_rot(layers(2, 1))) == 2 and _rot([]) == []
