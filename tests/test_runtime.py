"""C++ host runtime: paged KV block manager + continuous-batching scheduler (CPU)."""
import numpy as np
import pytest

from aws_k8s_ansible_provisioner_amd import _runtime_loader

rt = _runtime_loader.load()


def test_block_manager_alloc_free_and_prefix_cache():
    bm = rt.BlockManager(8, 4, True)
    assert bm.num_free == 8
    blocks = [bm.allocate() for _ in range(3)]
    assert len(set(blocks)) == 3 and bm.num_free == 5
    toks = list(range(100, 112))
    h0 = rt.BlockManager.hash_block(0, toks[0:4])
    h1 = rt.BlockManager.hash_block(h0, toks[4:8])
    bm.register_full(blocks[0], h0)
    bm.register_full(blocks[1], h1)
    bm.free_blocks(blocks)
    assert bm.num_free == 8  # cached blocks are evictable, counted free
    n, hit, hashes = bm.match_prefix(toks, 11)
    assert n == 8 and hit == blocks[:2] and hashes == [h0, h1]
    # a different first block breaks the chain
    n2, _, _ = bm.match_prefix([1] + toks[1:], 11)
    assert n2 == 0
    bm.free_blocks(hit)
    # exhaust the pool: evicts cached blocks (LRU), never hands out a block twice
    got = [bm.allocate() for _ in range(8)]
    assert sorted(got) == list(range(8))
    assert bm.allocate() == -1
    with pytest.raises(Exception):
        bm.free_blocks([got[0], got[0]])


def _bufs(max_seqs, cap_tokens, mb, tiles=256):
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


def _sched(num_blocks=64, bs=4, max_seqs=4, budget=16, max_len=64, prefix=True, G=2,
           tile_rows_short=0, short_rows=1024):
    c = rt.SchedConfig()
    c.max_num_seqs, c.max_num_batched_tokens, c.max_model_len = max_seqs, budget, max_len
    c.block_size, c.gqa_group, c.tile_rows, c.eos_id = bs, G, 64, 2
    c.tile_rows_short, c.short_rows = tile_rows_short, short_rows
    c.max_blocks_per_seq = max_len // bs
    return rt.Scheduler(c, num_blocks, prefix), _bufs(max_seqs, budget + max_seqs, max_len // bs)


def test_chunked_prefill_then_decode_and_slots():
    s, b = _sched(budget=8)
    s.add_request(1, list(range(10, 22)), 3, temperature=0.5, top_k=7, seed=99)  # 12 tokens
    i = s.schedule(b)
    assert i["is_prefill"] and i["num_tokens"] == 8 and i["num_samples"] == 0
    assert list(b["positions"][:8]) == list(range(8))
    bt = b["block_tables"][:16]
    slots = [bt[p // 4] * 4 + p % 4 for p in range(8)]
    assert list(b["slots"][:8]) == slots
    assert s.update(np.zeros(0, np.int64))[0] == []
    i = s.schedule(b)
    assert i["is_prefill"] and i["num_tokens"] == 4 and i["num_samples"] == 1
    assert b["logits_idx"][0] == 3 and b["top_k"][0] == 7 and b["seeds"][0] == 99
    assert b["temperature"][0] == pytest.approx(0.5) and b["steps"][0] == 0
    ids, toks, fin, first = s.update(np.array([55], np.int64))
    assert ids == [1] and toks == [55] and fin == [0] and first == [1]
    i = s.schedule(b)
    assert not i["is_prefill"] and i["num_seqs"] == 1 and i["num_tokens"] == 1
    assert b["input_ids"][0] == 55 and b["positions"][0] == 12 and b["seq_lens"][0] == 13
    assert b["steps"][0] == 1
    s.update(np.array([56], np.int64))
    s.schedule(b)
    ids, toks, fin, first = s.update(np.array([57], np.int64))
    assert fin == [1]  # length
    assert s.output_tokens(1) == [55, 56, 57]
    assert not s.has_work()


def test_prefill_tile_map_counts_gqa_rows():
    s, b = _sched(budget=64, max_len=128, G=4)
    s.add_request(1, list(range(3, 40)), 2)  # 37 tokens * 4 rows = 148 rows -> 3 tiles
    s.add_request(2, [5, 6], 2)               # 2 * 4 = 8 rows -> 1 tile
    i = s.schedule(b)
    assert i["num_tiles"] == 4
    # sorted by ascending causal work (keys seen by the tile's last row): seq 1's 2-token
    # tile, then seq 0's tiles ending at tokens 16, 32, 37 (the kernel runs the map back to front)
    assert list(b["tile_seq"][:4]) == [1, 0, 0, 0] and list(b["tile_row"][:4]) == [0, 0, 64, 128]
    assert list(b["q_start"][:3]) == [0, 37, 39]


def test_prefill_tile_rows_short_steps():
    """tile_rows_short: a step whose every prefill chunk has <= short_rows flattened q rows maps
    its tiles at the short granularity and reports it; a step with a longer chunk keeps
    tile_rows."""
    s2, b2 = _sched(budget=64, max_len=128, G=4, tile_rows_short=256, short_rows=160)
    s2.add_request(1, list(range(3, 40)), 2)  # 37 * 4 = 148 rows <= 160 -> one 256-row tile
    s2.add_request(2, [5, 6], 2)
    i = s2.schedule(b2)
    assert i["tile_rows"] == 256 and i["num_tiles"] == 2
    assert list(b2["tile_seq"][:2]) == [1, 0] and list(b2["tile_row"][:2]) == [0, 0]
    s3, b3 = _sched(budget=64, max_len=128, G=4, tile_rows_short=256, short_rows=100)
    s3.add_request(1, list(range(3, 40)), 2)  # 148 rows > 100 -> tile_rows (64)
    i = s3.schedule(b3)
    assert i["tile_rows"] == 64 and i["num_tiles"] == 3


def test_eos_stop_ids_and_min_tokens():
    s, b = _sched()
    s.add_request(1, [5, 6, 7], 10)  # eos=2 stops
    s.add_request(2, [5, 6, 8], 10, min_tokens=2)  # eos ignored before min_tokens
    s.add_request(3, [5, 6, 9], 10, stop_ids=[77])
    s.add_request(4, [5, 6, 10], 10, ignore_eos=True)
    s.schedule(b)
    ids, toks, fin, first = s.update(np.array([2, 2, 77, 2], np.int64))
    res = dict(zip(ids, fin))
    assert res[1] == 2 and res[2] == 0 and res[3] == 2 and res[4] == 0


def test_prefix_cache_hit_on_second_request():
    s, b = _sched(budget=64)
    p = list(range(20, 37))  # 17 tokens -> 4 full blocks
    s.add_request(1, p, 1)
    s.schedule(b)
    s.update(np.array([9], np.int64))
    s.add_request(2, p, 1)
    i = s.schedule(b)
    assert i["num_tokens"] == 1  # 16 cached tokens, only the last prompt token computed
    assert s.request_info(2)["num_cached"] == 16
    hits, queries = s.prefix_stats()
    assert hits == 16 and queries == 2 * 16  # tokens (vLLM's prefix-cache metric units)


def test_preemption_when_pool_exhausted():
    s, b = _sched(num_blocks=6, bs=4, max_seqs=4, budget=32, max_len=32)
    s.add_request(1, list(range(3, 11)), 12)  # 8 tokens = 2 blocks
    s.add_request(2, list(range(3, 11)) * 1, 12, stop_ids=[])
    s.add_request(3, list(range(13, 21)), 12)
    s.schedule(b)
    s.update(np.array([1, 1, 1], np.int64)[: 3])
    preempted = 0
    for _ in range(12):
        i = s.schedule(b)
        if i["num_seqs"] == 0:
            break
        preempted += i["num_preempted"]
        s.update(np.full(i["num_samples"], 4, np.int64))
    assert preempted >= 1 and s.total_preemptions >= 1
    # everything eventually finishes with all blocks returned
    for _ in range(200):
        if not s.has_work():
            break
        i = s.schedule(b)
        s.update(np.full(i["num_samples"], 4, np.int64))
    assert not s.has_work()
    assert s.num_free_blocks() == 6


def test_abort():
    s, b = _sched()
    s.add_request(1, [5, 6, 7], 10)
    s.add_request(2, [5, 6, 8], 10)
    assert s.abort_request(1)
    assert not s.abort_request(1)
    i = s.schedule(b)
    assert i["num_seqs"] == 1 and b["req_ids"][0] == 2


def test_mixed_step_runs_decodes_first_then_prefill_chunks():
    """Mixed batching: a running decode is scheduled in the same step as a newcomer's
    prefill chunk (decode rows lead; the tile map covers only the prefill rows)."""
    s, b = _sched(budget=16, bs=4, max_seqs=4, G=2)
    s.add_request(1, list(range(10, 18)), 8)
    i = s.schedule(b)
    assert i["is_prefill"] == 1 and i["num_decode"] == 0 and i["num_tokens"] == 8
    s.update(np.array([5], np.int64))
    s.add_request(2, list(range(40, 52)), 8)
    i = s.schedule(b)
    assert i["is_prefill"] == 1 and i["num_decode"] == 1
    assert i["num_seqs"] == 2 and i["num_tokens"] == 1 + 12
    assert list(b["req_ids"][:2]) == [1, 2]  # decode row first
    assert b["q_start"][1] == 1 and b["seq_lens"][0] == 9
    # tiles only for the prefill sequence (index 1): 12 tokens x G=2 rows / 64 -> one tile
    assert i["num_tiles"] == 1 and b["tile_seq"][0] == 1
    assert i["num_samples"] == 2 and list(b["logits_idx"][:2]) == [0, 12]
    s.update(np.array([6, 7], np.int64))
    i = s.schedule(b)  # nothing left to prefill: a pure decode step
    assert i["is_prefill"] == 0 and i["num_decode"] == 2 and i["num_tokens"] == 2


def test_prefill_first_policy_still_available():
    c = rt.SchedConfig()
    c.max_num_seqs, c.max_num_batched_tokens, c.max_model_len = 4, 16, 64
    c.block_size, c.gqa_group, c.tile_rows, c.eos_id, c.max_blocks_per_seq = 4, 2, 64, 2, 16
    c.mixed_batching = False
    s, b = rt.Scheduler(c, 64, True), _bufs(4, 20, 16)
    s.add_request(1, list(range(10, 18)), 8)
    s.schedule(b)
    s.update(np.array([5], np.int64))
    s.add_request(2, list(range(40, 52)), 8)
    i = s.schedule(b)
    assert i["is_prefill"] == 1 and i["num_decode"] == 0 and i["num_seqs"] == 1


def test_held_kv_expires_after_ttl():
    """P/D prefill side: KV held for a decode engine that never pulls it is freed once its
    TTL passes (no permanent leak), and free_held after expiry is a no-op."""
    c = rt.SchedConfig()
    c.max_num_seqs, c.max_num_batched_tokens, c.max_model_len = 4, 32, 64
    c.block_size, c.gqa_group, c.tile_rows, c.eos_id, c.max_blocks_per_seq = 4, 2, 64, 2, 16
    c.held_kv_ttl_s = 30.0
    s, b = rt.Scheduler(c, 32, False), _bufs(4, 36, 16)
    s.add_request(7, list(range(10, 22)), 1)
    s.set_hold_kv(7, True)
    s.schedule(b)
    s.update(np.array([5], np.int64))
    assert s.num_held == 1 and len(s.held_blocks(7)) == 3
    assert s.kv_usage() > 0
    assert s.expire_held(rt.Scheduler.now_s()) == 0  # not yet
    assert s.expire_held(rt.Scheduler.now_s() + 31.0) == 1
    assert s.num_held == 0 and s.kv_usage() == 0 and s.held_expired_total == 1
    s.free_held(7)  # late release after expiry: harmless
    assert s.kv_usage() == 0


def test_held_kv_in_transfer_survives_ttl_and_release():
    """A send that started owns its blocks: neither the TTL sweep nor a decode side's
    /kv/release (free_held) may recycle them while they are being packed; only the send's
    completion (finish_transfer) frees them (/kv/push vs expire_held race)."""
    c = rt.SchedConfig()
    c.max_num_seqs, c.max_num_batched_tokens, c.max_model_len = 4, 32, 64
    c.block_size, c.gqa_group, c.tile_rows, c.eos_id, c.max_blocks_per_seq = 4, 2, 64, 2, 16
    c.held_kv_ttl_s = 30.0
    s, b = rt.Scheduler(c, 32, False), _bufs(4, 36, 16)
    s.add_request(7, list(range(10, 22)), 1)
    s.set_hold_kv(7, True)
    s.schedule(b)
    s.update(np.array([5], np.int64))
    held = list(s.held_blocks(7))
    assert s.take_held(7) == held and s.num_held == 0 and s.num_in_transfer == 1
    free0 = s.num_free_blocks()
    assert s.expire_held(rt.Scheduler.now_s() + 999.0) == 0  # not TTL-tracked any more
    s.free_held(7)  # a late /kv/release from a decode side that gave up: no effect
    assert s.num_free_blocks() == free0 and s.kv_usage() > 0
    # a new prefill cannot be handed the blocks still being sent
    s.add_request(8, list(range(40, 60)), 1)
    i = s.schedule(b)
    assert not set(s.block_table(8)) & set(held), (s.block_table(8), held)
    s.update(np.zeros(i["num_samples"], np.int64) + 5)
    s.finish_transfer(7)
    s.finish_transfer(7)  # idempotent
    assert s.num_in_transfer == 0
    assert s.take_held(7) == []  # nothing held any more


def test_last_appended_counts_only_live_rows():
    """generation_tokens_total counts tokens actually appended: a lookahead row of a request
    that finished by EOS in the previous update is computed and discarded, not counted."""
    c = rt.SchedConfig()
    c.max_num_seqs, c.max_num_batched_tokens, c.max_model_len = 4, 64, 64
    c.block_size, c.gqa_group, c.tile_rows, c.eos_id, c.max_blocks_per_seq = 4, 2, 64, 2, 16
    s, b = rt.Scheduler(c, 64, False), _bufs(4, 68, 16)
    s.add_request(1, [10, 11, 12], 8)
    s.add_request(2, [20, 21, 22], 8)
    i = s.schedule(b)
    s.update(np.array([5, 5], np.int64))
    assert s.last_appended == 2
    i = s.schedule(b)  # pure decode, both rows
    assert i["num_seqs"] == 2 and not i["is_prefill"]
    b["src_rows"] = np.zeros(4, np.int64)
    la = s.schedule_lookahead(b)
    assert la["num_seqs"] == 2
    s.update(np.array([2, 5], np.int64))  # request 1 hits EOS (id 2)
    assert s.last_appended == 2
    s.update(np.array([7, 7], np.int64))  # lookahead: request 1's row is discarded
    assert s.last_appended == 1


def test_burst_backlog_stays_prefill_first_for_a_bounded_number_of_steps():
    """A prefill backlog larger than one step's budget (burst arrival) is drained
    prefill-first (TTFT) -- but decodes wait at most max_decode_stall_steps steps; once the
    backlog fits in a step, decodes and prefill chunks mix."""
    c = rt.SchedConfig()
    c.max_num_seqs, c.max_num_batched_tokens, c.max_model_len = 8, 16, 128
    c.block_size, c.gqa_group, c.tile_rows, c.eos_id, c.max_blocks_per_seq = 4, 2, 64, 2, 32
    c.max_decode_stall_steps = 3
    s, b = rt.Scheduler(c, 256, False), _bufs(8, 24, 32)
    s.add_request(1, list(range(10, 26)), 50)   # 16 tokens: fills step 1
    for k in range(2, 8):                        # 6 x 16 = 96 tokens queued behind it
        s.add_request(k, list(range(100 * k, 100 * k + 16)), 50)
    kinds = []
    for _ in range(8):
        i = s.schedule(b)
        kinds.append((i["is_prefill"], i["num_decode"]))
        s.update(np.zeros(i["num_samples"], np.int64) + 5)
    # step 1: pure prefill (nothing decoding); steps 2-4: backlog > budget -> prefill-first
    # while request 1 waits (3 stall steps); step 5: stall bound -> mixed; afterwards no run
    # of decode-stalling prefill steps is longer than the bound
    assert kinds[0] == (1, 0)
    assert kinds[1:4] == [(1, 0)] * 3
    assert kinds[4][0] == 1 and kinds[4][1] >= 1
    run = longest = 0
    for k in kinds[1:]:
        run = run + 1 if k[1] == 0 else 0
        longest = max(longest, run)
    assert longest <= 3


def _fake_model(b, info, req_of_row, prev=None):
    """Deterministic stand-in for the GPU step: the token sampled for a row depends on its
    input id, position and request; chained (lookahead) steps gather their input ids from
    the previous step's samples through src_rows, as the runner does on the device."""
    n, ns = info["num_tokens"], info["num_samples"]
    ids = b["input_ids"][:n].copy()
    if prev is not None:
        ids = prev[b["src_rows"][:n]]
    rows = b["logits_idx"][:ns]
    pos = b["positions"][:n]
    seq = b["req_ids"][:info["num_seqs"]]
    req = np.repeat(seq, np.diff(b["q_start"][:info["num_seqs"] + 1]))
    toks = (ids[rows] * 31 + pos[rows] * 7 + req[rows] * 5) % 97 + 3
    toks[(ids[rows] + pos[rows]) % 11 == 0] = 2  # EOS now and then
    for j in range(n):
        req_of_row.setdefault(int(req[j]), {})[int(pos[j])] = int(ids[j])
    return toks.astype(np.int64)


def _drive(lookahead, prompts, max_tokens, ignore_eos, num_blocks=256, max_seqs=4):
    s, b = _sched(num_blocks=num_blocks, max_seqs=max_seqs, budget=16, max_len=64)
    b["src_rows"] = np.zeros(max_seqs, np.int64)
    for i, p in enumerate(prompts):
        s.add_request(i + 1, p, max_tokens[i], 0, ignore_eos[i], [], stream=True)
    out = {i + 1: [] for i in range(len(prompts))}
    fed, inflight, n_look = {}, None, 0
    for _ in range(1000):
        if not s.has_work():
            break
        if inflight is None:
            info = s.schedule(b)
            toks = _fake_model(b, info, fed)
            if lookahead and not info["is_prefill"] and info["num_seqs"]:
                i2 = s.schedule_lookahead(b)
                if i2["num_seqs"]:
                    inflight = _fake_model(b, i2, fed, prev=toks)
                    n_look += 1
        else:
            toks = inflight
            i2 = s.schedule_lookahead(b)
            inflight = None
            if i2["num_seqs"]:
                inflight = _fake_model(b, i2, fed, prev=toks)
                n_look += 1
        ids, new, fin, _ = s.update(toks)
        for rid, tok, f in zip(ids, new, fin):
            if tok >= 0:
                out[rid].append(tok)
            if f:
                s.release(rid)  # what the engine does after delivering the finish
    assert not s.has_work()
    assert s.kv_usage() == 0.0
    return out, fed, n_look


def test_decode_lookahead_matches_synchronous_scheduling():
    """Async (lookahead) decode scheduling produces exactly the synchronous token streams:
    rows finished by EOS while their next step was in flight are discarded, rows that the
    in-flight token ends by length are left out, and every computed row fed the model the
    right input id at the right position."""
    rng = np.random.default_rng(0)
    prompts = [list(rng.integers(3, 90, size=int(k))) for k in (5, 9, 3, 12, 7, 4)]
    max_tokens = [6, 11, 1, 9, 14, 3]
    ignore_eos = [True, False, True, False, False, True]
    ref, _, n0 = _drive(False, prompts, max_tokens, ignore_eos)
    got, fed, n1 = _drive(True, prompts, max_tokens, ignore_eos)
    assert n0 == 0 and n1 > 5
    assert got == ref
    for rid, toks in got.items():
        full = list(prompts[rid - 1]) + toks
        for pos, tok in fed[rid].items():
            if pos < len(full) - 1:  # rows past the end were computed and discarded
                assert tok == full[pos], (rid, pos)


def test_decode_lookahead_declines_when_work_waits():
    s, b = _sched(num_blocks=64, max_seqs=4, budget=16, max_len=64)
    b["src_rows"] = np.zeros(4, np.int64)
    s.add_request(1, [5, 6, 7], 8, 0, True, [])
    info = s.schedule(b)
    assert info["is_prefill"]
    assert s.schedule_lookahead(b)["num_seqs"] == 0  # never after a prefill step
    s.update(np.array([9], np.int64))
    info = s.schedule(b)
    assert not info["is_prefill"]
    s.add_request(2, [5, 6], 8, 0, True, [])  # a waiting request needs a normal step
    assert s.schedule_lookahead(b)["num_seqs"] == 0  # (a free sequence slot could admit it)
    s.update(np.array([9], np.int64))
    s.abort_request(2)
    s.schedule(b)
    la = s.schedule_lookahead(b)
    assert la["num_seqs"] == 1 and b["src_rows"][0] == 0 and b["positions"][0] == 5
    assert s.schedule_lookahead(b)["num_seqs"] == 0  # at most one step ahead


def test_decode_lookahead_continues_while_the_queue_cannot_be_admitted():
    """Every sequence slot taken: waiting requests could not be admitted by a normal step
    either, so lookahead continues -- until the in-flight step ends a row by length."""
    s, b = _sched(num_blocks=64, max_seqs=2, budget=16, max_len=64)
    b["src_rows"] = np.zeros(2, np.int64)
    s.add_request(1, [5, 6, 7], 3, 0, True, [])
    s.add_request(2, [8, 9], 8, 0, True, [])
    s.add_request(3, [4, 4], 4, 0, True, [])  # waits: max_num_seqs = 2
    assert s.schedule(b)["is_prefill"]
    s.update(np.array([11, 12], np.int64))
    assert not s.schedule(b)["is_prefill"]  # both decode; request 1 has 1 of 3 tokens
    la = s.schedule_lookahead(b)
    assert la["num_seqs"] == 2  # queue non-empty, but no slot is free
    s.update(np.array([13, 14], np.int64))
    # request 1's in-flight token is its 3rd: it ends by length -> a normal step admits 3
    assert s.schedule_lookahead(b)["num_seqs"] == 0


try:
    from hypothesis import given, settings
    from hypothesis import strategies as st_
except ImportError:  # pragma: no cover
    given = None

if given is not None:
    @settings(max_examples=60, deadline=None)
    @given(st_.lists(st_.tuples(st_.integers(1, 20), st_.integers(1, 16), st_.booleans()),
                     min_size=1, max_size=9),
           st_.integers(0, 10 ** 6), st_.sampled_from([2, 4, 8]), st_.sampled_from([24, 48, 256]))
    def test_decode_lookahead_property(reqs, seed, max_seqs, num_blocks):
        """Random request mixes (queueing behind max_num_seqs, KV pools small enough to
        preempt, EOS finishes while a lookahead step is in flight): the lookahead loop emits
        exactly the synchronous loop's token streams and frees every block."""
        rng = np.random.default_rng(seed)
        prompts = [list(rng.integers(3, 90, size=n)) for n, _, _ in reqs]
        mt = [m for _, m, _ in reqs]
        ie = [e for _, _, e in reqs]
        ref_out, _, _ = _drive(False, prompts, mt, ie, num_blocks, max_seqs)
        got, _, _ = _drive(True, prompts, mt, ie, num_blocks, max_seqs)
        assert got == ref_out


def test_v_tail_slots_follow_each_sequence_and_return_to_the_pool():
    """V-tail slots (AttnParams.v_tail): every token row carries its sequence's slot, a slot
    is stable while the sequence runs, and finish / abort / preemption hand it back."""
    c = rt.SchedConfig()
    c.max_num_seqs, c.max_num_batched_tokens, c.max_model_len = 4, 32, 32
    c.block_size, c.gqa_group, c.tile_rows, c.eos_id = 4, 2, 64, 2
    c.max_blocks_per_seq, c.num_tail_slots = 8, 8
    s = rt.Scheduler(c, 6, True)
    b = _bufs(4, 36, 8)
    b["tail_slot"] = np.full(36, -7, np.int32)
    s.add_request(1, list(range(3, 11)), 12)
    s.add_request(2, list(range(13, 20)), 12)
    s.add_request(3, list(range(23, 31)), 12)
    i = s.schedule(b)
    seen = {}
    for r in range(i["num_seqs"]):
        a, e = int(b["q_start"][r]), int(b["q_start"][r + 1])
        ts = set(b["tail_slot"][a:e].tolist())
        assert len(ts) == 1 and min(ts) >= 0
        seen[int(b["req_ids"][r])] = ts.pop()
    assert len(set(seen.values())) == len(seen)  # distinct slots
    s.update(np.full(i["num_samples"], 4, np.int64))
    preempted = 0
    for _ in range(200):
        if not s.has_work():
            break
        i = s.schedule(b)
        preempted += i["num_preempted"]
        for r in range(i["num_seqs"]):
            rid, t = int(b["req_ids"][r]), int(b["tail_slot"][int(b["q_start"][r])])
            assert t >= 0
            if preempted == 0:  # stable while it runs (a recomputed sequence may move)
                assert seen.setdefault(rid, t) == t
        s.update(np.full(i["num_samples"], 4, np.int64))
    assert preempted >= 1  # the 6-block pool cannot hold all three: one was recomputed
    assert s.num_free_tail_slots == 8
    # abort hands the slot back too; a scheduler without slots stages -1
    s.add_request(9, [5, 6, 7], 4)
    s.schedule(b)
    assert s.num_free_tail_slots == 7 and s.abort_request(9)
    assert s.num_free_tail_slots == 8
    s0, b0 = _sched()
    b0["tail_slot"] = np.zeros(20, np.int32)
    s0.add_request(1, [5, 6, 7], 4)
    s0.schedule(b0)
    assert b0["tail_slot"][:3].tolist() == [-1, -1, -1]


def test_prefill_tile_map_sorted_by_causal_work_with_context():
    """The tile map is sorted by ascending causal work -- keys seen by the tile's last row,
    context included -- so a continued chunk's tiles (prior context) come after a fresh short
    prompt's; the prefill attention kernel walks the map back to front (longest first)."""
    s, b = _sched(budget=40, max_len=128, G=2)
    s.add_request(1, list(range(3, 63)), 2)   # 60 tokens: 40 now, 20 in the next step
    i = s.schedule(b)
    assert i["num_tiles"] == 2  # 80 rows / 64
    s.update(np.zeros(0, np.int64))
    s.add_request(2, [5, 6, 7], 2)            # fresh 3-token prompt
    i = s.schedule(b)
    n = i["num_tiles"]
    seqs = list(b["tile_seq"][:n])
    rows = list(b["tile_row"][:n])
    qs, sl = list(b["q_start"][:3]), list(b["seq_lens"][:2])
    work = []
    for t in range(n):
        q = qs[seqs[t] + 1] - qs[seqs[t]]
        work.append(sl[seqs[t]] - q + min(q, -(-(rows[t] + 64) // 2)))
    assert work == sorted(work) and work == [3, 60]  # fresh 3-token tile, then 40 + 20 keys
    assert sorted(zip(seqs, rows)) == sorted(set(zip(seqs, rows)))  # no tile lost or doubled
