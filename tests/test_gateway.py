"""Gateway + endpoint picker: scoring, prefix affinity, P/D pairing, failover, and an
end-to-end run of the reference smoke test (llm-d-test.yaml) through the gateway in
front of two real CPU engine servers."""
import asyncio
import json
import socket
import threading
import time

import aiohttp
import pytest
import uvicorn
from aiohttp import web

from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig
from aws_k8s_ansible_provisioner_amd.gateway.picker import (Endpoint, EndpointPicker,
                                                            PickerConfig, parse_prometheus,
                                                            prefix_hashes)
from aws_k8s_ansible_provisioner_amd.gateway.server import Gateway, _parse_dns, _parse_targets
from aws_k8s_ansible_provisioner_amd.server.api_server import build_app

MODEL = "Qwen/Qwen3-0.6B"


def test_picker_prefers_least_loaded_and_kv_headroom():
    p = EndpointPicker([Endpoint("a"), Endpoint("b"), Endpoint("c")])
    p.update_metrics("a", running=10, waiting=5, kv=0.9)
    p.update_metrics("b", running=1, waiting=0, kv=0.2)
    p.update_metrics("c", running=4, waiting=1, kv=0.5)
    assert p.pick("x").url == "b"
    p.mark_failure("b", hard=True)
    assert p.pick("x").url == "c"


def test_picker_prefix_affinity():
    p = EndpointPicker([Endpoint("a"), Endpoint("b")], PickerConfig(w_prefix=5.0))
    for u in "ab":
        p.update_metrics(u, 0, 0, 0.0)
    doc = "shared system prompt " * 40
    first = p.pick(doc + " q1").url
    # same long prefix -> same endpoint even when it is slightly busier
    p.update_metrics(first, running=2, waiting=0, kv=0.1)
    assert p.pick(doc + " q2").url == first
    assert len(prefix_hashes(doc, 64)) == len(doc) // 64


def test_picker_pd_pairs():
    eps = [Endpoint("p1", "prefill"), Endpoint("d1", "decode"), Endpoint("m1", "both")]
    p = EndpointPicker(eps, PickerConfig(pd_threshold_chars=100))
    pre, dec = p.pick_pd("y" * 200)
    assert pre.url == "p1" and dec.url == "d1"
    pre, dec = p.pick_pd("short")
    assert pre is None and dec.url in ("m1", "d1")
    pre, dec = p.pick_pd("y" * 200, pd_ok=False)  # n > 1 / several prompts: monolithic
    assert pre is None


def test_picker_pd_pairs_only_within_a_transfer_group():
    """Two `pd` pods behind one gateway: a prefill is never paired with the other pod's
    decode rank (its RCCL send could not pair with that recv -> both would hang)."""
    p = EndpointPicker([], PickerConfig(pd_threshold_chars=10), seed=3)
    p.set_endpoints([("http://10.0.0.1:8000", "prefill"), ("http://10.0.0.1:8001", "decode"),
                     ("http://10.0.0.2:8000", "prefill"), ("http://10.0.0.2:8001", "decode")])
    for u in [e.url for e in p.endpoints()]:
        p.update_metrics(u, 0, 0, 0.0)
    seen = set()
    for i in range(40):
        # load one pod's decode heavily: an independent pick would mix pods
        p.update_metrics("http://10.0.0.1:8001", running=50, waiting=20, kv=0.9)
        pre, dec = p.pick_pd(f"{i} " + "z" * 50)
        assert pre.group == dec.group
        assert pre.url.split(":")[1] == dec.url.split(":")[1]
        seen.add(pre.group)
    assert seen == {"10.0.0.2"}  # the pair on the idle pod wins on combined score
    # a group that lost its decode endpoint cannot serve P/D; the other group still can
    p.mark_failure("http://10.0.0.2:8001", hard=True)
    pre, dec = p.pick_pd("q" * 50)
    assert pre.url == "http://10.0.0.1:8000" and dec.url == "http://10.0.0.1:8001"
    p.mark_failure("http://10.0.0.1:8000", hard=True)
    pre, dec = p.pick_pd("q" * 50)  # no complete group: monolithic on a decode endpoint
    assert pre is None and dec.url == "http://10.0.0.1:8001"


def test_picker_pd_prefers_ipc_decode():
    """among valid P/D pairs the gateway prefers one whose decode endpoint
    pulls KV by hipIpc (akap:kv_transport_ipc) over a slightly less loaded send/recv pair."""
    p = EndpointPicker([], PickerConfig(pd_threshold_chars=10), seed=1)
    p.set_endpoints([("http://a:8000", "prefill", "g"), ("http://b:8001", "decode", "g"),
                     ("http://c:8001", "decode", "g")])
    p.update_metrics("http://a:8000", 0, 0, 0.0)
    p.update_metrics("http://b:8001", running=2, waiting=0, kv=0.2, kv_ipc=True)
    p.update_metrics("http://c:8001", 0, 0, 0.0, kv_ipc=False)
    for _ in range(10):
        pre, dec = p.pick_pd("x" * 40)
        assert dec.url == "http://b:8001"
    p.update_metrics("http://b:8001", running=2, waiting=0, kv=0.2, kv_ipc=False)
    pre, dec = p.pick_pd("x" * 40)
    assert dec.url == "http://c:8001"


def test_rccl_transport_parse():
    from aws_k8s_ansible_provisioner_amd.parallel.kv_transfer import transport_from_rccl_log

    log = ("host:1:2 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC\n"
           "host:1:2 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC\n")
    assert transport_from_rccl_log(log) == "P2P"
    assert transport_from_rccl_log(log + "x NCCL INFO Channel 02/0 : 0 -> 1 via SHM/direct/direct") == "SHM"
    assert transport_from_rccl_log("NCCL INFO Channel 00/0 : 0[0] -> 1[0] [send] via NET/Socket/0") == "NET"
    assert transport_from_rccl_log("nothing") == "unknown"


def test_parsers():
    m = parse_prometheus('# HELP x\nvllm:num_requests_running{model_name="m"} 3.0\n'
                         'vllm:num_requests_running{model_name="n"} 2\nbad line\n')
    assert m["vllm:num_requests_running"] == 5.0
    assert _parse_targets("a:8000@prefill,http://b:9/,c:1@decode:g7") == [
        ("http://a:8000", "prefill", ""), ("http://b:9", "both", ""),
        ("http://c:1", "decode", "g7")]
    assert _parse_dns("svc.ns.svc.cluster.local:8000@decode") == [
        ("svc.ns.svc.cluster.local", 8000, "decode", "")]
    # two-pod P/D: both Deployments' services carry one named P/D group
    assert _parse_dns("a-prefill:8000@prefill:akap-pd,a-decode:8000@decode:akap-pd") == [
        ("a-prefill", 8000, "prefill", "akap-pd"), ("a-decode", 8000, "decode", "akap-pd")]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Uvicorn(threading.Thread):
    def __init__(self, app, port):
        super().__init__(daemon=True)
        self.server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port,
                                                    log_level="error"))

    def run(self):
        self.server.run()


@pytest.fixture(scope="module")
def two_engines():
    servers, urls = [], []
    for i in range(2):
        ecfg = EngineConfig(model="tiny-qwen3", served_model_name=MODEL, device="cpu",
                            max_model_len=256, max_num_seqs=8, max_num_batched_tokens=64,
                            block_size=32, num_gpu_blocks=128, seed=i)
        app, _ = build_app(ecfg)
        port = _free_port()
        t = _Uvicorn(app, port)
        t.start()
        servers.append(t)
        urls.append(f"http://127.0.0.1:{port}")
    for u in urls:
        for _ in range(200):
            try:
                import urllib.request
                urllib.request.urlopen(u + "/health", timeout=1)
                break
            except Exception:
                time.sleep(0.05)
    yield urls
    for t in servers:
        t.server.should_exit = True


def test_gateway_end_to_end_reference_smoke(two_engines):
    async def run():
        gw = Gateway([(u, "both") for u in two_engines] + [("http://127.0.0.1:9", "both")], [],
                     scrape_interval=0.2)
        app = gw.app()
        runner = web.AppRunner(app)
        await runner.setup()
        port = _free_port()
        site = web.TCPSite(runner, "127.0.0.1", port)
        await site.start()
        base = f"http://127.0.0.1:{port}"
        try:
            await asyncio.sleep(0.5)
            async with aiohttp.ClientSession() as s:
                # llm-d-test.yaml:32-59 -- GET /v1/models through the gateway
                async with s.get(base + "/v1/models") as r:
                    text = await r.text()
                assert MODEL in text
                # llm-d-test.yaml:61-78 -- POST /v1/completions through the gateway
                for _ in range(6):
                    async with s.post(base + "/v1/completions",
                                      json={"model": MODEL, "prompt": "Who are you?"}) as r:
                        assert r.status == 200
                        j = await r.json()
                        assert j["choices"][0]["text"] is not None
                # streaming passthrough
                async with s.post(base + "/v1/chat/completions",
                                  json={"messages": [{"role": "user", "content": "hi"}],
                                        "max_tokens": 3, "stream": True}) as r:
                    body = await r.text()
                assert body.rstrip().endswith("data: [DONE]")
                async with s.get(base + "/health") as r:
                    h = await r.json()
                assert len(h["endpoints"]) == 2  # the dead :9 endpoint was ejected
                async with s.get(base + "/metrics") as r:
                    m = await r.text()
                assert "akap_gateway_requests_total" in m
            served = {e.url: e.served for e in gw.picker.endpoints()}
            assert sum(served.values()) >= 7
        finally:
            await runner.cleanup()

    asyncio.run(run())


def test_gateway_api_controller_programs_status():
    """The gateway's Gateway API controller (class akap) against a fake API server: the
    GatewayClass is accepted, the Gateway gets status.addresses[0] = its Service's ClusterIP
    (tier 1 of /root/reference/llm-d-test.yaml:14-26's lookup) plus Accepted/Programmed, the
    HTTPRoute's parent is accepted; a second pass writes nothing new; a class owned by
    another controller is left alone."""
    import asyncio
    import json as _json

    import aiohttp as _aiohttp
    from aiohttp import web as _web

    from aws_k8s_ansible_provisioner_amd.gateway.k8s_controller import (CONTROLLER_NAME,
                                                                         GatewayController)

    gw_api = "/apis/gateway.networking.k8s.io/v1"
    state = {
        "gc": {"metadata": {"name": "akap", "generation": 1},
               "spec": {"controllerName": CONTROLLER_NAME}},
        "gw": {"metadata": {"name": "llm-d-inference-gateway", "generation": 2},
               "spec": {"gatewayClassName": "akap",
                        "listeners": [{"name": "http", "protocol": "HTTP", "port": 80}]}},
        "other": {"metadata": {"name": "other-gw", "generation": 1},
                  "spec": {"gatewayClassName": "istio", "listeners": []}},
        "rt": {"metadata": {"name": "llm-d-inference-gateway", "generation": 1},
               "spec": {"parentRefs": [{"name": "llm-d-inference-gateway"}]}},
    }
    patches = []

    async def gc(req):
        return _web.json_response(state["gc"])

    async def gws(req):
        return _web.json_response({"items": [state["gw"], state["other"]]})

    async def rts(req):
        return _web.json_response({"items": [state["rt"]]})

    async def svc(req):
        if req.match_info["name"] != "llm-d-inference-gateway":
            return _web.json_response({}, status=404)
        return _web.json_response({"spec": {"clusterIP": "10.96.7.7"}})

    async def patch(req):
        assert req.headers["Content-Type"] == "application/merge-patch+json"
        assert req.headers["Authorization"] == "Bearer tok"
        body = _json.loads(await req.text())
        patches.append((req.path, body))
        kind = req.match_info["kind"]
        key = {"gatewayclasses": "gc", "gateways": "gw", "httproutes": "rt"}[kind]
        state[key]["status"] = body["status"]
        return _web.json_response(state[key])

    async def run():
        app = _web.Application()
        app.router.add_get(gw_api + "/gatewayclasses/akap", gc)
        app.router.add_get(gw_api + "/namespaces/llm-d/gateways", gws)
        app.router.add_get(gw_api + "/namespaces/llm-d/httproutes", rts)
        app.router.add_get("/api/v1/namespaces/llm-d/services/{name}", svc)
        app.router.add_patch(gw_api + "/{kind}/{name}/status", patch)
        app.router.add_patch(gw_api + "/namespaces/llm-d/{kind}/{name}/status", patch)
        runner = _web.AppRunner(app)
        await runner.setup()
        site = _web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        ctl = GatewayController("llm-d", api=f"http://127.0.0.1:{port}", token="tok")
        try:
            async with _aiohttp.ClientSession() as s:
                first = await ctl.reconcile(s)
                n1 = len(patches)
                await ctl.reconcile(s)
                n2 = len(patches)
                state["gc"]["spec"]["controllerName"] = "example.com/other"
                third = await ctl.reconcile(s)
        finally:
            await runner.cleanup()
        return first, n1, n2, third

    first, n1, n2, third = asyncio.run(run())
    assert first["gatewayclass"] and first["gateways"] == {"llm-d-inference-gateway": "10.96.7.7"}
    assert first["routes"] == ["llm-d-inference-gateway"]
    st = state["gw"]["status"]
    assert st["addresses"] == [{"type": "IPAddress", "value": "10.96.7.7"}]
    assert {c["type"] for c in st["conditions"]} == {"Accepted", "Programmed"}
    assert st["listeners"][0]["attachedRoutes"] == 1
    assert "status" not in state["other"]  # another class: untouched
    assert state["rt"]["status"]["parents"][0]["controllerName"] == CONTROLLER_NAME
    # level-triggered and idempotent: the second pass only re-asserts the route parent
    assert n2 - n1 == 1, patches[n1:]
    assert third["gatewayclass"] is False and not third["gateways"]
