"""Fault injection (SURVEY §5 "Failure detection": kill an engine mid-stream, drop a KV
transfer, lose a replica behind the gateway).  CPU engines, real HTTP servers."""
import asyncio
import socket
import threading
import time
import urllib.request

import aiohttp
import pytest
import uvicorn
from aiohttp import web
from fastapi.testclient import TestClient

from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
from aws_k8s_ansible_provisioner_amd.gateway.server import Gateway
from aws_k8s_ansible_provisioner_amd.server.api_server import build_app


def _cfg(**kw):
    base = dict(model="tiny-qwen3", served_model_name="m", device="cpu", max_model_len=128,
                max_num_seqs=4, max_num_batched_tokens=64, block_size=32, num_gpu_blocks=64)
    base.update(kw)
    return EngineConfig(**base)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_engine_crash_fails_requests_and_health():
    app, ae = build_app(_cfg())
    calls = {"n": 0}
    orig = ae.engine.runner.execute

    def flaky(info):
        calls["n"] += 1
        if calls["n"] > 2:
            raise RuntimeError("injected GPU fault")
        return orig(info)

    ae.engine.runner.execute = flaky
    with TestClient(app) as c:
        assert c.get("/health").status_code == 200
        r = c.post("/v1/completions", json={"prompt": "hello", "max_tokens": 20,
                                            "ignore_eos": True})
        assert r.status_code == 500 and "injected GPU fault" in r.text
        assert c.get("/health").status_code == 503   # readiness probe now fails
        # new requests are refused fast instead of hanging
        r = c.post("/v1/completions", json={"prompt": "x", "max_tokens": 2})
        assert r.status_code == 500
        # streaming requests get the error in-band and a terminated stream
        r = c.post("/v1/completions", json={"prompt": "x", "max_tokens": 2, "stream": True})
        assert "error" in r.text and r.text.rstrip().endswith("data: [DONE]")


def test_dropped_kv_transfer_errors_and_frees_blocks():
    app, ae = build_app(_cfg())
    ae.kv_agent = object()  # decode role; the transfer fails before any data moves
    eng = ae.engine
    free0 = eng.sched.num_free_blocks()
    kvp = {"transfer_id": 7, "prompt_token_ids": list(range(3, 40)), "first_token": 5,
           "remote_rank": 0, "num_blocks": 3,
           "remote_url": f"http://127.0.0.1:{_free_port()}"}  # prefill pod is gone
    with TestClient(app) as c:
        r = c.post("/v1/completions", json={"prompt": "ignored", "max_tokens": 8,
                                            "kv_transfer_params": kvp})
        assert r.status_code >= 500
        for _ in range(100):
            if eng.sched.num_free_blocks() == free0:
                break
            time.sleep(0.02)
        assert eng.sched.num_free_blocks() == free0, "reserved KV blocks leaked"
        # the engine is still healthy and serves monolithic requests
        assert c.get("/health").status_code == 200
        r = c.post("/v1/completions", json={"prompt": "hi", "max_tokens": 3})
        assert r.status_code == 200


class _Server(threading.Thread):
    def __init__(self, app, port):
        super().__init__(daemon=True)
        self.server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port,
                                                    log_level="error"))

    def run(self):
        self.server.run()


def test_gateway_survives_replica_loss_mid_run():
    urls, servers = [], []
    for i in range(2):
        app, _ = build_app(_cfg(seed=i))
        port = _free_port()
        t = _Server(app, port)
        t.start()
        servers.append(t)
        urls.append(f"http://127.0.0.1:{port}")
    for u in urls:
        for _ in range(200):
            try:
                urllib.request.urlopen(u + "/health", timeout=1)
                break
            except Exception:
                time.sleep(0.05)

    async def run():
        gw = Gateway([(u, "both") for u in urls], [], scrape_interval=0.1)
        runner = web.AppRunner(gw.app())
        await runner.setup()
        gport = _free_port()
        await web.TCPSite(runner, "127.0.0.1", gport).start()
        ok = 0
        try:
            await asyncio.sleep(0.3)
            async with aiohttp.ClientSession() as s:
                for k in range(12):
                    if k == 4:  # kill replica 0 mid-run
                        servers[0].server.should_exit = True
                        await asyncio.sleep(0.5)
                    async with s.post(f"http://127.0.0.1:{gport}/v1/completions",
                                      json={"prompt": f"q{k}", "max_tokens": 2}) as r:
                        ok += r.status == 200
            ep = {e.url: e for e in gw.picker.endpoints()}
            assert not ep[urls[0]].healthy
        finally:
            await runner.cleanup()
        return ok

    try:
        assert asyncio.run(run()) == 12
    finally:
        for t in servers:
            t.server.should_exit = True


class _FakeIpcAgent:
    """P/D prefill-side agent stand-in: records what /kv/push would send."""
    is_gpu = True
    broken = None

    def __init__(self):
        self.sent = []

    def ipc_meta(self):
        return {"handles": []}

    def send_blocks(self, blocks, dst, on_done=None):
        self.sent.append((list(blocks), dst))
        if on_done:
            on_done()


def test_kv_push_uses_server_lease_record_not_client_blocks():
    """a /kv/push fallback after /kv/lease ships the blocks this server
    leased, never a client-supplied list (forged ids would read past the cache or ship
    other requests' KV)."""
    app, ae = build_app(_cfg())
    eng = ae.engine
    held = {5: [1, 2], 6: [3]}
    finished = []
    eng.held_blocks = lambda t: list(held.get(t, []))
    eng.take_held = lambda t: held.pop(t, [])
    eng.finish_transfer = lambda t: finished.append(t)
    ag = _FakeIpcAgent()
    ae.kv_agent = ag
    with TestClient(app) as c:
        r = c.post("/kv/lease", json={"transfer_ids": [5]})
        assert r.status_code == 200 and r.json()["blocks"] == [[1, 2]]
        # forged list for a leased transfer: refused, nothing sent
        r = c.post("/kv/push", json={"transfer_ids": [5], "leased_blocks": [[10 ** 9]],
                                     "dst_rank": 1})
        assert r.status_code == 409 and not ag.sent
        # a transfer that was never leased: refused
        r = c.post("/kv/push", json={"transfer_ids": [6], "leased_blocks": [[3]],
                                     "dst_rank": 1})
        assert r.status_code == 404 and not ag.sent
        # the genuine fallback ships the recorded blocks once
        r = c.post("/kv/push", json={"transfer_ids": [5], "leased_blocks": [[1, 2]],
                                     "dst_rank": 1})
        assert r.status_code == 200 and ag.sent == [([1, 2], 1)] and finished == [5]
        r = c.post("/kv/push", json={"transfer_ids": [5], "leased_blocks": [[1, 2]],
                                     "dst_rank": 1})
        assert r.status_code == 404  # the lease was consumed


def test_kv_agent_rejects_out_of_range_block_ids():
    import torch

    from aws_k8s_ansible_provisioner_amd.parallel.kv_transfer import KVTransferAgent

    kv = torch.zeros(2, 2, 8, 64, dtype=torch.bfloat16)
    ag = KVTransferAgent(kv)
    assert ag._ids([0, 7]).tolist() == [0, 7]
    for bad in ([8], [-1], [0, 100]):
        with pytest.raises(IndexError):
            ag._ids(bad)
    with pytest.raises(IndexError):
        ag.gather([9])


def test_collective_timeout_word_fails_step_not_tokens():
    """a custom IPC collective that timed out inside a replayed decode
    step only sets the kernels' error word.  The runner copies it to the host behind the
    step and checks it before any token is used: the request errors, /health goes 503, and
    no token of that step reaches the client.  (CPU engine; the word is injected.)"""
    import torch

    from aws_k8s_ansible_provisioner_amd.engine.model_runner import ModelRunner
    from aws_k8s_ansible_provisioner_amd.parallel.comm import CollectiveTimeout

    with pytest.raises(CollectiveTimeout):
        ModelRunner._check_err(torch.tensor([1], dtype=torch.int32))
    ModelRunner._check_err(torch.tensor([0], dtype=torch.int32))
    ModelRunner._check_err(None)
    with pytest.raises(CollectiveTimeout):
        ModelRunner.wait_decode((None, torch.tensor([5, 6]), torch.tensor([1], dtype=torch.int32)))

    app, ae = build_app(_cfg())
    runner = ae.engine.runner
    steps = {"n": 0}

    def probe(slot):
        steps["n"] += 1
        # the third step's collectives "time out" (sticky from then on, like the kernel word)
        return torch.tensor([1 if steps["n"] >= 3 else 0], dtype=torch.int32)

    runner._err_probe = probe
    with TestClient(app) as c:
        r = c.post("/v1/completions", json={"prompt": "hello", "max_tokens": 16,
                                            "ignore_eos": True})
        assert r.status_code == 500 and "timed out" in r.text
        assert c.get("/health").status_code == 503
