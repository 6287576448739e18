"""The hipIpc mapping of a peer cache is bounded: a hipIpcOpenMemHandle that never returns
(seen for a large export mapped by a second importer on one device, profiles/
r4_pd_1p2d_one_gpu.log) must not block the caller; the peer falls back to the p2p transport."""
import base64
import time

import pytest
import torch

from aws_k8s_ansible_provisioner_amd import ops
from aws_k8s_ansible_provisioner_amd.parallel import kv_transfer
from aws_k8s_ansible_provisioner_amd.parallel.kv_transfer import (KVIpcOpenTimeout,
                                                                  KVTransferAgent, bounded_call)


def test_bounded_call_returns_value_and_raises():
    assert bounded_call(lambda: 41 + 1, 5.0, "quick") == 42
    with pytest.raises(ValueError):
        bounded_call(lambda: (_ for _ in ()).throw(ValueError("boom")), 5.0, "raises")
    t0 = time.monotonic()
    with pytest.raises(KVIpcOpenTimeout):
        bounded_call(lambda: time.sleep(30), 0.3, "stuck open")
    assert time.monotonic() - t0 < 5.0


def test_connect_ipc_times_out_then_fails_fast(monkeypatch):
    kv = torch.zeros(2, 2, 4, 64, dtype=torch.bfloat16)
    ag = KVTransferAgent(kv)
    try:
        ag.ipc_open_timeout_s = 0.3
        calls = []

        def stuck(blob, dev):
            calls.append(1)
            time.sleep(30)

        monkeypatch.setattr(ops, "ipc_open", stuck)
        meta = {"segments": [{"blob": base64.b64encode(b"x" * 80).decode(), "planes": 4}],
                "planes": 4, "nblocks": 4, "block_elems": 64, "plane_stride": 256}
        t0 = time.monotonic()
        with pytest.raises(KVIpcOpenTimeout):
            ag.connect_ipc(meta)
        assert time.monotonic() - t0 < 5.0
        # the failed peer is remembered: no second (stuck) open, an immediate error
        with pytest.raises(KVIpcOpenTimeout):
            ag.connect_ipc(meta)
        assert len(calls) == 1 and not ag.ipc_connected
        # an fp8 (byte) cache refuses V-tail jobs (no V tail in fp8 caches)
        ag8 = KVTransferAgent(torch.zeros(2, 2, 4, 128, dtype=torch.uint8))
        assert ag8.byte_cache and ag8.block_elems == 64
        ag8.peers["k"] = ([0] * 4, 4, [])
        with pytest.raises(ValueError):
            ag8.pull([(0, 0)], 1, 32, 4, tail_jobs=[(0, 0, 1, 0)], peer="k")
        ag8.peers = {}
        ag8.close()
    finally:
        ag.close()


def test_default_timeout_env(monkeypatch):
    assert kv_transfer.IPC_OPEN_TIMEOUT_S > 0


def test_segmented_kv_cache_views_and_packing():
    """A large cache is several allocations (layer ranges, AKAP_KV_SEGMENT_GIB): the per-layer
    views, the p2p pack/unpack over every segment's planes and the plane address table of the
    IPC pull all see the same [2L planes] cache as one allocation would."""
    from aws_k8s_ansible_provisioner_amd import ops
    from aws_k8s_ansible_provisioner_amd.models.config import get_config
    from aws_k8s_ansible_provisioner_amd.models.transformer import DecoderLM

    m = DecoderLM(get_config("tiny-qwen3"), device="cpu", max_model_len=256)
    L = m.cfg.num_layers
    one = m.allocate_kv_cache(16, 32)
    per_layer = one[0].numel() * one.element_size()
    segs = m.allocate_kv_segments(16, 32, max_segment_bytes=per_layer)  # one layer each
    assert len(segs) == L and all(t.shape[0] == 1 for t in segs)
    torch.manual_seed(0)
    for l in range(L):
        segs[l].copy_(torch.randn(segs[l].shape).to(segs[l].dtype))
        one[l].copy_(segs[l][0])
    ks1, vs1 = m.cache_views(one, 32)
    ks2, vs2 = m.cache_views(segs, 32)
    assert all(torch.equal(a, b) for a, b in zip(ks1, ks2))
    assert all(torch.equal(a, b) for a, b in zip(vs1, vs2))
    a1, a2 = KVTransferAgent(one), KVTransferAgent(segs)
    try:
        ids = torch.tensor([3, 0, 7], dtype=torch.int32)
        assert a2.num_planes == 2 * L and a2.nbytes(3) == a1.nbytes(3)
        assert torch.equal(a1._gather(ids), a2._gather(ids))
        buf = torch.randn(2 * L, 2, a2.block_elems).to(torch.bfloat16)
        dst = torch.tensor([5, 9], dtype=torch.int32)
        a1._scatter(buf, dst)
        a2._scatter(buf, dst)
        assert all(torch.equal(one[l], segs[l][0]) for l in range(L))
        tab = ops.plane_table(a2.planes_list)
        assert len(tab) == 2 * L and tab[1] - tab[0] == segs[0][0, 0].numel() * 2
    finally:
        a1.close()
        a2.close()


def test_ipc_safe_alloc_bytes_rule():
    """The bundled ROCm 7.0.2 runtime hangs in hipIpcOpenMemHandle when bit 31 of the
    allocation size is set (profiles/r6_ipc_import_sweep.md: 1.5 / 5 / 8 / 9.5 / 36 GiB map,
    2 / 2.5 / 6.6 GiB hang).  The KV allocator pads such sizes to the next 4 GiB multiple."""
    from aws_k8s_ansible_provisioner_amd.models.transformer import ipc_safe_alloc_bytes

    G = 2**30
    for gib in (1.5, 5, 8, 9.5, 36):  # measured to map: unchanged (2 MiB rounding only)
        assert ipc_safe_alloc_bytes(int(gib * G)) == int(gib * G)
    for gib, want in ((2, 4), (2.5, 4), (6.6, 8), (31.7, 32), (86, 88)):  # measured / r4-r5 hangs
        r = ipc_safe_alloc_bytes(int(gib * G))
        assert r == want * G and not r & (1 << 31)
    assert ipc_safe_alloc_bytes(1) == 2 << 20  # the caching allocator's 2 MiB rounding
    for n in (3 * G + 5, 7 * G - 1, 123456789012):
        r = ipc_safe_alloc_bytes(n)
        assert r >= n and not r & (1 << 31) and r - n < 2 * G + (2 << 20)


def test_kv_segment_layers_avoid_padding():
    """Layers per segment: the count in [max/2, max] with the fewest padding bytes.  Llama-3-8B
    at the round-5 1P:1D size (32 layers, ~3.17 GiB each, 32 GiB cap): 10 layers per segment
    would make 31.7 GiB allocations (bit 31 set); the choice needs no padding at all."""
    from aws_k8s_ansible_provisioner_amd.models.transformer import (ipc_safe_alloc_bytes,
                                                                  kv_segment_layers)

    G = 2**30
    per_layer = int(3.17 * G) // (2 << 20) * (2 << 20)
    lps = kv_segment_layers(32, per_layer, 32 * G)
    assert 5 < lps <= 10
    pad = sum(ipc_safe_alloc_bytes(min(lps, 32 - l0) * per_layer) - min(lps, 32 - l0) * per_layer
              for l0 in range(0, 32, lps))
    assert pad == 0
    assert kv_segment_layers(32, per_layer, 32 * G, ipc_safe=False) == 10
    assert kv_segment_layers(4, 10 * G, 32 * G) in (2, 3)  # never below half the max
    assert kv_segment_layers(28, G // 16, 32 * G) == 28  # 1.75 GiB: one unpadded segment
    assert kv_segment_layers(28, G // 8, 32 * G) == 15  # 3.5 GiB (bit 31): 1.875 + 1.625 GiB
