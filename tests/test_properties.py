"""Property-based (hypothesis) and randomized stress tests of the host runtime and of the
op references ("hypothesis shape fuzzing"; §5: "deterministic stress tests for
scheduler / KV allocator").  All CPU."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from aws_k8s_ansible_provisioner_amd import _runtime_loader, ops
from aws_k8s_ansible_provisioner_amd.ops import reference as ref
from aws_k8s_ansible_provisioner_amd.utils import chat_template, tracing

rt = _runtime_loader.load()
FAST = settings(max_examples=40, deadline=None,
                suppress_health_check=[HealthCheck.too_slow])


# ----------------------------------------------------------------------------- allocator
@FAST
@given(st.lists(st.tuples(st.sampled_from(["alloc", "free", "reg", "match"]),
                          st.integers(0, 10 ** 6)), max_size=200),
       st.integers(1, 24), st.booleans())
def test_block_manager_never_double_allocates(opsq, nblocks, prefix):
    bm = rt.BlockManager(nblocks, 4, prefix)
    held: list[int] = []           # blocks we own a reference to (may repeat: shared hits)
    for op, r in opsq:
        if op == "alloc":
            b = bm.allocate()
            if b == -1:
                # only legal when every block is referenced
                assert len(set(held)) == nblocks
            else:
                assert b not in held, "allocator returned a referenced block"
                held.append(b)
        elif op == "free" and held:
            b = held.pop(r % len(held))
            bm.free_blocks([b])
        elif op == "reg" and held and prefix:
            b = held[r % len(held)]
            bm.register_full(b, rt.BlockManager.hash_block(0, [r % 97, 1, 2, 3]))
        elif op == "match":
            toks = [r % 97, 1, 2, 3, 9]
            n, hit, _ = bm.match_prefix(toks, 5)
            assert n == 4 * len(hit)
            held.extend(hit)
        assert 0 <= bm.num_free <= nblocks
        assert bm.num_free >= nblocks - len(set(held)) - 0
    bm.free_blocks(held)
    assert bm.num_free == nblocks


# ----------------------------------------------------------------------------- scheduler
def _bufs(max_seqs, cap_tokens, mb, tiles=512):
    return {
        "input_ids": np.zeros(cap_tokens, np.int64), "positions": np.zeros(cap_tokens, np.int64),
        "slots": np.zeros(cap_tokens, np.int64), "seq_lens": np.zeros(max_seqs, np.int32),
        "q_start": np.zeros(max_seqs + 1, np.int32),
        "block_tables": np.zeros(max_seqs * mb, np.int32),
        "tile_seq": np.zeros(tiles, np.int32), "tile_row": np.zeros(tiles, np.int32),
        "logits_idx": np.zeros(max_seqs, np.int64), "req_ids": np.zeros(max_seqs, np.int64),
        "sample_mask": np.zeros(max_seqs, np.int32),
        "temperature": np.zeros(max_seqs, np.float32), "top_p": np.zeros(max_seqs, np.float32),
        "top_k": np.zeros(max_seqs, np.int32), "seeds": np.zeros(max_seqs, np.int64),
        "steps": np.zeros(max_seqs, np.int32),
    }


def _check_batch(i, b, cfg):
    ns, nt = i["num_seqs"], i["num_tokens"]
    assert 0 < ns <= cfg["max_seqs"]
    assert nt <= max(cfg["budget"], cfg["max_seqs"])
    qs = b["q_start"][:ns + 1]
    assert qs[0] == 0 and qs[ns] == nt and np.all(np.diff(qs) >= 1)
    slots = b["slots"][:nt]
    assert len(set(slots.tolist())) == nt, "two tokens write the same KV slot"
    mb = cfg["max_len"] // cfg["bs"]
    for s in range(ns):
        L = int(b["seq_lens"][s])
        assert 0 < L <= cfg["max_len"]
        row = b["block_tables"][s * mb:(s + 1) * mb]
        for t in range(qs[s], qs[s + 1]):
            p = int(b["positions"][t])
            assert p < L
            assert slots[t] == row[p // cfg["bs"]] * cfg["bs"] + p % cfg["bs"]


@settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.integers(0, 2 ** 31 - 1), st.booleans(), st.integers(6, 40))
def test_scheduler_random_workload_invariants(seed, prefix, nblocks):
    rng = np.random.default_rng(seed)
    cfg = dict(max_seqs=4, budget=24, max_len=48, bs=4)
    c = rt.SchedConfig()
    c.max_num_seqs, c.max_num_batched_tokens, c.max_model_len = 4, 24, 48
    c.block_size, c.gqa_group, c.tile_rows, c.eos_id = 4, 2, 64, 2
    c.max_blocks_per_seq = 12
    s = rt.Scheduler(c, nblocks, prefix)
    b = _bufs(4, 24, 12)
    max_tok = {}
    outs = {}
    nreq = int(rng.integers(1, 12))
    shared = list(rng.integers(3, 50, size=8))
    for r in range(1, nreq + 1):
        plen = int(rng.integers(1, 20))
        prompt = (shared[:plen] if rng.random() < 0.5 else
                  list(rng.integers(3, 50, size=plen)))
        mt = int(rng.integers(1, 48 - plen))
        s.add_request(r, [int(x) for x in prompt], mt,
                      stop_ids=[int(rng.integers(3, 50))] if rng.random() < 0.3 else [])
        max_tok[r] = mt
    aborted = set()
    for _ in range(2000):
        if not s.has_work():
            break
        if rng.random() < 0.02:
            victim = int(rng.integers(1, nreq + 1))
            if s.abort_request(victim):
                aborted.add(victim)
        i = s.schedule(b)
        if i["num_seqs"]:
            _check_batch(i, b, cfg)
        toks = rng.integers(2, 50, size=i["num_samples"]).astype(np.int64)
        ids, new, fin, first = s.update(toks)  # also flushes scheduler-ended requests
        for rid, f in zip(ids, fin):
            if f:
                outs[rid] = s.output_tokens(rid)
                s.release(rid)
    assert not s.has_work()
    for rid, o in outs.items():
        assert len(o) <= max_tok[rid]
    assert s.num_free_blocks() == nblocks


# ----------------------------------------------------------------------------- op references
@FAST
@given(st.integers(1, 40), st.integers(1, 8), st.integers(1, 3), st.sampled_from([4, 16, 64]),
       st.integers(0, 10 ** 6))
def test_moe_align_reference_properties(T, E, K, block, seed):
    K = min(K, E)
    g = torch.Generator().manual_seed(seed)
    ids = torch.stack([torch.randperm(E, generator=g)[:K] for _ in range(T)]).to(torch.int32)
    s, off, npad = ops.moe_align(ids, E, block)
    n = T * K
    assert off[0] == 0 and int(npad) == int(off[-1]) <= s.numel()
    real = s[: int(npad)]
    real = real[real < n]
    assert sorted(real.tolist()) == list(range(n))
    for e in range(E):
        seg = s[off[e]:off[e + 1]]
        assert (off[e + 1] - off[e]) % block == 0
        assert all(int(ids.reshape(-1)[x]) == e for x in seg.tolist() if x < n)


@FAST
@given(st.integers(1, 6), st.sampled_from([(2, 1), (4, 2), (4, 4), (8, 1)]),
       st.sampled_from([32, 64]), st.integers(0, 10 ** 6))
def test_paged_attention_reference_block_table_invariance(B, heads, BS, seed):
    """Permuting physical blocks (and the tables with them) must not change the output."""
    Hq, Hkv = heads
    D = 32
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(1, 3 * BS, (B,), generator=g)
    mb = 3
    nb = B * mb
    kc = torch.randn(nb, Hkv, BS, D, generator=g)
    vc = torch.randn(nb, Hkv, BS // 8, D, 8, generator=g)
    tables = torch.arange(nb, dtype=torch.int32).view(B, mb)
    q_len = torch.minimum(lens, torch.randint(1, 5, (B,), generator=g))
    q_start = torch.cat([torch.zeros(1, dtype=torch.int32), q_len.cumsum(0).to(torch.int32)])
    q = torch.randn(int(q_start[-1]), Hq, D, generator=g)
    out1 = ref.paged_attention(q, kc, vc, tables, lens, q_start, D ** -0.5)
    perm = torch.randperm(nb, generator=g)
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(nb)
    out2 = ref.paged_attention(q, kc[perm], vc[perm], inv[tables.long()].to(torch.int32), lens,
                               q_start, D ** -0.5)
    assert torch.allclose(out1, out2, atol=1e-5)


@FAST
@given(st.integers(2, 300), st.floats(0.05, 2.0), st.integers(0, 50), st.floats(0.1, 1.0),
       st.integers(0, 10 ** 6))
def test_sampler_reference_support_properties(V, temp, k, p, seed):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(3, V, generator=g)
    toks, lps = ref.sample(logits, torch.full((3,), temp), torch.full((3,), k, dtype=torch.int32),
                           torch.full((3,), p), torch.arange(3), torch.zeros(3))
    for i in range(3):
        t = int(toks[i])
        assert 0 <= t < V
        if 0 < k < V:
            assert logits[i, t] >= torch.topk(logits[i], k).values[-1]
        assert float(lps[i]) <= 1e-6


# ----------------------------------------------------------------------------- misc
@FAST
@given(st.text(max_size=80))
def test_traceparent_parser_total(s):
    tid, sid = tracing.parse_traceparent(s)
    assert (tid is None) == (sid is None)
    if tid is not None:
        assert tracing.parse_traceparent(tracing.make_traceparent(tid, sid)) == (tid, sid)


@FAST
@given(st.lists(st.fixed_dictionaries({
    "role": st.sampled_from(["system", "user", "assistant"]),
    "content": st.text(max_size=40)}), min_size=1, max_size=6),
    st.sampled_from(["phi", "opt", "default"]))
def test_chat_templates_render_any_conversation(msgs, name):
    out = chat_template.render(msgs, chat_template.BUILTIN[name], True)
    assert isinstance(out, str)
    for m in msgs:
        if m["role"] != "system" or name == "default":
            assert m["content"] in out


@settings(max_examples=200, deadline=None)
@given(st.lists(st.integers(0, 151935), max_size=300), st.booleans())
def test_byte_tokenizer_decode_matches_reference_loop(ids, skip):
    """The vectorised ByteTokenizer.decode equals the per-id definition: specials skipped,
    bytes [3, 259) verbatim, anything else -> the printable placeholder 33 + id % 94."""
    from aws_k8s_ansible_provisioner_amd.utils.tokenizer import ByteTokenizer

    tk = ByteTokenizer(151936, 151643, 151645)
    ids = ids + [151643, 151645, 0][: len(ids) % 4]
    out = bytearray()
    for i in ids:
        if skip and i in (151643, 151645, 0):
            continue
        b = i - 3
        out.append(b if 0 <= b < 256 else 33 + i % 94)
    assert tk.decode(ids, skip_special=skip) == out.decode("utf-8", errors="replace")
    assert tk.decode(np.asarray(ids), skip_special=skip) == tk.decode(ids, skip_special=skip)
