"""OTLP trace export + W3C trace-context propagation (SURVEY §5 tracing row).

A local HTTP "collector" stands in for the OTel collector's :4318 receiver and records
the OTLP/JSON bodies; the tests check span structure, parenting across the gateway ->
engine hop, and the gen_ai.* attributes."""
import asyncio
import http.server
import json
import threading
import time

import aiohttp
import pytest
from aiohttp import web

from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine
from aws_k8s_ansible_provisioner_amd.utils import tracing


class _Collector:
    def __init__(self):
        self.bodies = []
        outer = self

        class H(http.server.BaseHTTPRequestHandler):
            def do_POST(self):
                n = int(self.headers.get("Content-Length", 0))
                outer.bodies.append((self.path, json.loads(self.rfile.read(n))))
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.end_headers()
                self.wfile.write(b"{}")

            def log_message(self, *a):
                pass

        self.srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.port = self.srv.server_address[1]
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def spans(self):
        out = []
        for path, b in self.bodies:
            assert path == "/v1/traces"
            for rs in b["resourceSpans"]:
                svc = {a["key"]: a["value"] for a in rs["resource"]["attributes"]}
                for ss in rs["scopeSpans"]:
                    for sp in ss["spans"]:
                        sp = dict(sp)
                        sp["service"] = svc["service.name"]["stringValue"]
                        sp["attrs"] = {a["key"]: list(a["value"].values())[0]
                                       for a in sp["attributes"]}
                        out.append(sp)
        return out

    def close(self):
        self.srv.shutdown()


@pytest.fixture()
def collector():
    c = _Collector()
    tr = tracing.configure(f"http://127.0.0.1:{c.port}", service_name="test-engine",
                           flush_interval=0.1)
    yield c, tr
    tracing.configure(None)
    c.close()


def test_traceparent_roundtrip():
    tid, sid = tracing.new_trace_id(), tracing.new_span_id()
    hdr = tracing.make_traceparent(tid, sid)
    assert tracing.parse_traceparent(hdr) == (tid, sid)
    assert tracing.parse_traceparent("garbage") == (None, None)
    assert tracing.parse_traceparent("00-" + "0" * 32 + "-" + "1" * 16 + "-01") == (None, None)
    assert tracing.parse_traceparent(None) == (None, None)


def test_export_batches_and_drops_when_collector_down():
    tr = tracing.OTLPTracer("http://127.0.0.1:9", flush_interval=60, timeout=0.5)
    tr.record("x", time.time(), time.time())
    tr.flush()
    assert tr.dropped == 1 and tr.exported == 0
    tr.shutdown()


def _engine():
    return LLMEngine(EngineConfig(model="tiny-qwen3", device="cpu", max_model_len=128,
                                  max_num_seqs=4, max_num_batched_tokens=64, block_size=32,
                                  num_gpu_blocks=64), log=lambda *a: None)


def test_engine_emits_request_spans_with_parent(collector):
    c, tr = collector
    eng = _engine()
    tid, sid = tracing.new_trace_id(), tracing.new_span_id()
    eng.add_request("r1", "hello world", SamplingParams(max_tokens=5, ignore_eos=True),
                    traceparent=tracing.make_traceparent(tid, sid))
    eng.add_request("r2", "untraced", SamplingParams(max_tokens=3, ignore_eos=True))
    while eng.has_unfinished():
        eng.step()
    tr.flush()
    spans = c.spans()
    by_name = {}
    for s in spans:
        by_name.setdefault(s["name"], []).append(s)
    roots = by_name["llm_request"]
    assert len(roots) == 2
    r1 = [s for s in roots if s["attrs"]["gen_ai.request.id"] == "r1"][0]
    assert r1["traceId"] == tid and r1["parentSpanId"] == sid
    assert r1["service"] == "test-engine"
    assert r1["attrs"]["gen_ai.usage.completion_tokens"] == "5"
    assert r1["attrs"]["gen_ai.response.finish_reason"] == "length"
    assert float(r1["attrs"]["gen_ai.latency.time_to_first_token"]) >= 0
    r2 = [s for s in roots if s["attrs"]["gen_ai.request.id"] == "r2"][0]
    assert r2["traceId"] != tid and "parentSpanId" not in r2
    kids = [s for s in spans if s.get("parentSpanId") == r1["spanId"]]
    assert sorted(k["name"] for k in kids) == ["decode", "prefill"]
    for k in kids:
        assert int(k["startTimeUnixNano"]) >= int(r1["startTimeUnixNano"])
        assert int(k["endTimeUnixNano"]) <= int(r1["endTimeUnixNano"])


def test_gateway_propagates_trace_to_engine(collector):
    import socket

    import uvicorn

    from aws_k8s_ansible_provisioner_amd.gateway.server import Gateway
    from aws_k8s_ansible_provisioner_amd.server.api_server import build_app

    c, tr = collector

    def free_port():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        return p

    ecfg = EngineConfig(model="tiny-qwen3", served_model_name="m", device="cpu",
                        max_model_len=128, max_num_seqs=4, max_num_batched_tokens=64,
                        block_size=32, num_gpu_blocks=64)
    app, _ = build_app(ecfg)
    eport = free_port()
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=eport, log_level="error"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    import urllib.request
    for _ in range(200):
        try:
            urllib.request.urlopen(f"http://127.0.0.1:{eport}/health", timeout=1)
            break
        except Exception:
            time.sleep(0.05)
    tid, sid = tracing.new_trace_id(), tracing.new_span_id()

    async def run():
        gw = Gateway([(f"http://127.0.0.1:{eport}", "both")], [], scrape_interval=0.2)
        runner = web.AppRunner(gw.app())
        await runner.setup()
        gport = free_port()
        await web.TCPSite(runner, "127.0.0.1", gport).start()
        try:
            await asyncio.sleep(0.3)
            async with aiohttp.ClientSession() as s:
                async with s.post(f"http://127.0.0.1:{gport}/v1/completions",
                                  json={"prompt": "hi", "max_tokens": 3},
                                  headers={"traceparent": tracing.make_traceparent(tid, sid)}
                                  ) as r:
                    assert r.status == 200
        finally:
            await runner.cleanup()

    try:
        asyncio.run(run())
    finally:
        server.should_exit = True
    tr.flush()
    spans = c.spans()
    gw = [s for s in spans if s["name"] == "gateway.route"]
    assert len(gw) == 1 and gw[0]["traceId"] == tid and gw[0]["parentSpanId"] == sid
    assert gw[0]["attrs"]["http.status_code"] == "200"
    req = [s for s in spans if s["name"] == "llm_request"]
    assert len(req) == 1
    assert req[0]["traceId"] == tid and req[0]["parentSpanId"] == gw[0]["spanId"]
