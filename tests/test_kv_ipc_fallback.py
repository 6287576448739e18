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
        meta = {"blob": base64.b64encode(b"x" * 80).decode(), "planes": 4, "nblocks": 4,
                "block_elems": 64, "plane_stride": 256}
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
        ag8.peers["k"] = (1, 4, 256)
        with pytest.raises(ValueError):
            ag8.pull([(0, 0)], 1, 32, 4, tail_jobs=[(0, 0, 1, 0)], peer="k")
        ag8.peers = {}
        ag8.close()
    finally:
        ag.close()


def test_default_timeout_env(monkeypatch):
    assert kv_transfer.IPC_OPEN_TIMEOUT_S > 0
