"""Inference gateway: OpenAI-compatible HTTP front door that routes every request to a
model-server pod chosen by the endpoint picker (gateway/picker.py).

Deployed as Service ``llm-d-inference-gateway`` (label app.kubernetes.io/name=
llm-d-inference-gateway, port 80) -- the address llm-d-test.yaml:14-26 resolves.

* endpoint discovery: a static list (``--endpoints url[@role],...``) and/or a headless
  Service DNS name re-resolved every few seconds (``--dns host:port[@role]``);
* health + load: every endpoint's /metrics is scraped (vllm:num_requests_running,
  vllm:num_requests_waiting, vllm:gpu_cache_usage_perc) on a short period;
* routing: least-loaded + KV headroom + prefix affinity; P/D: long prompts are
  prefilled on a prefill pod (max_tokens=1, kv_transfer_params.do_remote_decode) and
  decoded on a decode pod that pulls the KV cache over RCCL;
* failures: a connect error marks the endpoint down and the request is retried once on
  another endpoint (before any byte was streamed to the client).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import socket
import time
from typing import Optional
from urllib.parse import urlparse

import aiohttp
from aiohttp import web

from ..utils import tracing
from ..utils.metrics import Counter, Gauge, Histogram, LAT_BUCKETS, Registry
from .picker import Endpoint, EndpointPicker, PickerConfig, parse_prometheus


class Gateway:
    def __init__(self, static: list[tuple], dns: list[tuple[str, int, str]],
                 cfg: Optional[PickerConfig] = None, scrape_interval: float = 1.0,
                 request_timeout: float = 600.0):
        """static: (url, role[, P/D group]) tuples; dns: (host, port, role[, group])."""
        self.static = static
        self.dns = dns
        self.picker = EndpointPicker([], cfg)
        self.picker.set_endpoints(static)
        self.scrape_interval = scrape_interval
        self.timeout = aiohttp.ClientTimeout(total=request_timeout, sock_connect=5)
        self.session: Optional[aiohttp.ClientSession] = None
        self._tasks: list[asyncio.Task] = []
        self.reg = Registry()
        self.m_req = self.reg.add(Counter("akap_gateway_requests_total", "Routed requests",
                                          ("endpoint", "code", "route")))
        self.m_lat = self.reg.add(Histogram("akap_gateway_request_seconds", "Gateway latency",
                                            LAT_BUCKETS, ("route",)))
        self.m_up = self.reg.add(Gauge("akap_gateway_endpoint_up", "Endpoint health", ("endpoint", "role")))
        self.m_pd_fallback = self.reg.add(Counter(
            "akap_gateway_pd_fallback_total",
            "P/D requests served monolithically after a failed KV hand-off", ()))
        self.m_pd = self.reg.add(Counter("akap_gateway_pd_requests_total",
                                         "Requests served disaggregated", ()))
        # Gateway API controller for our GatewayClass (gateway/k8s_controller.py), in-cluster
        self.controller = None

    # ---------------------------------------------------------------- lifecycle
    async def start(self, app=None) -> None:
        self.session = aiohttp.ClientSession(timeout=self.timeout)
        await self.refresh_dns()
        self._tasks.append(asyncio.create_task(self._scrape_loop()))
        if self.dns:
            self._tasks.append(asyncio.create_task(self._dns_loop()))
        if self.controller is not None:
            self._tasks.append(asyncio.create_task(self.controller.run()))

    async def stop(self, app=None) -> None:
        for t in self._tasks:
            t.cancel()
        if self.session:
            await self.session.close()

    async def refresh_dns(self) -> None:
        found = list(self.static)
        loop = asyncio.get_running_loop()
        for host, port, role, group in self.dns:
            try:
                infos = await loop.getaddrinfo(host, port, type=socket.SOCK_STREAM)
                for ip in sorted({i[4][0] for i in infos}):
                    # P/D group: the pod IP by default (a pod's prefill :8000 and decode :8001
                    # ranks); a named group for two-pod P/D, where prefill and decode are
                    # separate Deployments whose servers form KV channels on demand
                    found.append((f"http://{ip}:{port}", role, group or ip))
            except OSError:
                pass
        self.picker.set_endpoints(found)

    async def _dns_loop(self) -> None:
        while True:
            await asyncio.sleep(5.0)
            await self.refresh_dns()

    async def scrape_once(self) -> None:
        async def one(e: Endpoint):
            try:
                async with self.session.get(e.url + "/metrics",
                                            timeout=aiohttp.ClientTimeout(total=2)) as r:
                    if r.status != 200:
                        raise aiohttp.ClientError(f"status {r.status}")
                    m = parse_prometheus(await r.text())
                self.picker.update_metrics(e.url, m.get("vllm:num_requests_running", 0.0),
                                           m.get("vllm:num_requests_waiting", 0.0),
                                           m.get("vllm:gpu_cache_usage_perc", 0.0),
                                           kv_broken=m.get("akap:kv_channel_broken", 0.0) > 0,
                                           kv_ipc=m.get("akap:kv_transport_ipc", 0.0) > 0)
            except (aiohttp.ClientError, asyncio.TimeoutError, OSError):
                self.picker.mark_failure(e.url)
            self.m_up.set(1.0 if e.healthy else 0.0, endpoint=e.url, role=e.role)

        await asyncio.gather(*[one(e) for e in self.picker.endpoints()])

    async def _scrape_loop(self) -> None:
        while True:
            await self.scrape_once()
            await asyncio.sleep(self.scrape_interval)

    # ---------------------------------------------------------------- proxy
    @staticmethod
    def _prompt_text(body: dict) -> str:
        if "messages" in body:
            parts = []
            for m in body.get("messages") or []:
                c = m.get("content", "")
                parts.append(c if isinstance(c, str) else json.dumps(c))
            return "\n".join(parts)
        p = body.get("prompt", "")
        return p if isinstance(p, str) else json.dumps(p)

    async def _forward(self, request: web.Request, ep: Endpoint, path: str, body: dict,
                       stream: bool, headers: Optional[dict] = None) -> web.StreamResponse:
        ep.inflight += 1
        try:
            async with self.session.post(ep.url + path, json=body, headers=headers) as up:
                if not stream or up.status != 200:
                    data = await up.read()
                    return web.Response(body=data, status=up.status,
                                        content_type=up.content_type or "application/json")
                resp = web.StreamResponse(status=200, headers={
                    "Content-Type": "text/event-stream", "Cache-Control": "no-cache"})
                await resp.prepare(request)
                async for chunk in up.content.iter_any():
                    await resp.write(chunk)
                await resp.write_eof()
                return resp
        finally:
            ep.inflight -= 1

    async def handle_generate(self, request: web.Request) -> web.StreamResponse:
        with tracing.Span("gateway.route", request.headers.get("traceparent"),
                          attributes={"http.route": request.path}) as span:
            resp = await self._route(request, span)
            span.attributes["http.status_code"] = resp.status
            span.error = resp.status >= 500
            return resp

    async def _route(self, request: web.Request, span) -> web.StreamResponse:
        t0 = time.time()
        path = request.path
        try:
            body = await request.json()
        except Exception:
            return web.json_response({"object": "error", "message": "invalid JSON"}, status=400)
        stream = bool(body.get("stream"))
        text = self._prompt_text(body)
        headers = {"traceparent": span.traceparent}
        tried: set[str] = set()
        # P/D hands ONE prefilled sequence to the decode pod: single prompt, n == 1
        p_ = body.get("prompt")
        pd_ok = (body.get("n") in (None, 1) and
                 not (isinstance(p_, list) and p_ and not isinstance(p_[0], int)))
        orig = body
        for attempt in range(2):
            pre, dec = self.picker.pick_pd(text, pd_ok)
            if dec is None or dec.url in tried:
                cands = [e for e in self.picker.endpoints() if e.healthy and e.url not in tried
                         and e.role in ("both", "decode")]
                if not cands:
                    break
                dec = cands[0]
            span.attributes["akap.endpoint"] = dec.url
            span.attributes["akap.attempt"] = attempt
            try:
                body = orig
                if pre is not None:
                    span.attributes["akap.prefill_endpoint"] = pre.url
                    body = await self._prefill_remote(pre, path, orig, headers)
                    self.m_pd.inc()
                resp = await self._forward(request, dec, path, body, stream, headers)
                if (pre is not None and resp.status >= 500 and attempt == 0
                        and isinstance(resp, web.Response)):
                    # KV hand-off failed on the decode pod (it released the prefill's held
                    # KV): serve this request monolithically instead
                    self.m_pd_fallback.inc()
                    pd_ok = False
                    body = orig
                    resp = await self._forward(request, dec, path, orig, stream, headers)
                self.m_req.inc(endpoint=dec.url, code=str(resp.status), route=path)
                self.m_lat.observe(time.time() - t0, route=path)
                return resp
            except (aiohttp.ClientConnectionError, asyncio.TimeoutError, OSError):
                self.picker.mark_failure(dec.url, hard=True)
                tried.add(dec.url)
        self.m_req.inc(endpoint="none", code="503", route=path)
        return web.json_response({"object": "error", "message": "no healthy model server",
                                  "type": "ServiceUnavailable"}, status=503)

    async def _prefill_remote(self, pre: Endpoint, path: str, body: dict,
                              headers: Optional[dict] = None) -> dict:
        """P/D step 1: prefill on `pre` (1 token), keep its KV for the decode pod."""
        pbody = dict(body)
        pbody["max_tokens"] = 1
        pbody["stream"] = False
        pbody.pop("stream_options", None)
        pbody["kv_transfer_params"] = {"do_remote_decode": True}
        pre.inflight += 1
        try:
            async with self.session.post(pre.url + path, json=pbody, headers=headers) as r:
                j = await r.json()
        finally:
            pre.inflight -= 1
        out = dict(body)
        if isinstance(j, dict) and j.get("kv_transfer_params"):
            kvp = dict(j["kv_transfer_params"])
            kvp["remote_url"] = pre.url
            out["kv_transfer_params"] = kvp
        return out

    async def handle_models(self, request: web.Request) -> web.Response:
        seen, data = set(), []
        for e in self.picker.endpoints():
            if not e.healthy:
                continue
            try:
                async with self.session.get(e.url + "/v1/models") as r:
                    j = await r.json()
                for m in j.get("data", []):
                    if m["id"] not in seen:
                        seen.add(m["id"])
                        data.append(m)
            except (aiohttp.ClientError, asyncio.TimeoutError, OSError, ValueError):
                self.picker.mark_failure(e.url)
        return web.json_response({"object": "list", "data": data})

    async def handle_health(self, request: web.Request) -> web.Response:
        up = [e.url for e in self.picker.endpoints() if e.healthy]
        return web.json_response({"status": "ok" if up else "degraded", "endpoints": up},
                                 status=200 if up else 503)

    async def handle_metrics(self, request: web.Request) -> web.Response:
        return web.Response(text=self.reg.render(), content_type="text/plain")

    async def handle_endpoints(self, request: web.Request) -> web.Response:
        return web.json_response([e.__dict__ for e in self.picker.endpoints()])

    def app(self) -> web.Application:
        app = web.Application(client_max_size=64 * 2**20)
        app.router.add_post("/v1/completions", self.handle_generate)
        app.router.add_post("/v1/chat/completions", self.handle_generate)
        app.router.add_get("/v1/models", self.handle_models)
        app.router.add_get("/health", self.handle_health)
        app.router.add_get("/metrics", self.handle_metrics)
        app.router.add_get("/debug/endpoints", self.handle_endpoints)
        app.on_startup.append(self.start)
        app.on_cleanup.append(self.stop)
        return app


def _parse_targets(spec: str) -> list[tuple[str, str, str]]:
    """url[@role[:group]],...  (group: P/D transfer group; default the URL's host)."""
    out = []
    for item in filter(None, (s.strip() for s in spec.split(","))):
        url, _, rg = item.partition("@")
        role, _, group = rg.partition(":")
        if "://" not in url:
            url = "http://" + url
        out.append((url.rstrip("/"), role or "both", group))
    return out


def _parse_dns(spec: str) -> list[tuple[str, int, str, str]]:
    """host:port[@role[:group]],...  (group: P/D group of every resolved endpoint; default the
    endpoint's own IP, i.e. P/D pairs only inside one pod)."""
    out = []
    for item in filter(None, (s.strip() for s in spec.split(","))):
        hp, _, rg = item.partition("@")
        role, _, group = rg.partition(":")
        u = urlparse("//" + hp)
        out.append((u.hostname, u.port or 8000, role or "both", group))
    return out


def main(argv=None) -> None:
    ap = argparse.ArgumentParser("akap-gateway")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=80)
    ap.add_argument("--endpoints", default="", help="url[@role],... (role: both|prefill|decode)")
    ap.add_argument("--dns", default="",
                    help="headless-service-host:port[@role[:group]],... (group: two-pod P/D)")
    ap.add_argument("--scrape-interval", type=float, default=1.0)
    ap.add_argument("--pd-threshold-chars", type=int, default=512)
    ap.add_argument("--w-prefix", type=float, default=2.0)
    ap.add_argument("--otlp-traces-endpoint", default=None)
    ap.add_argument("--gateway-controller", default="auto", choices=["auto", "on", "off"],
                    help="reconcile Gateway/HTTPRoute status for GatewayClass --gateway-class "
                         "(auto: when running in a cluster with a service-account token)")
    ap.add_argument("--gateway-class", default="akap")
    ap.add_argument("--namespace", default=os.environ.get("POD_NAMESPACE", "llm-d"))
    a = ap.parse_args(argv)
    tracing.configure(a.otlp_traces_endpoint, service_name=os.environ.get(
        "OTEL_SERVICE_NAME", "akap-gateway"))
    cfg = PickerConfig(pd_threshold_chars=a.pd_threshold_chars, w_prefix=a.w_prefix)
    gw = Gateway(_parse_targets(a.endpoints), _parse_dns(a.dns), cfg, a.scrape_interval)
    from . import k8s_controller

    if a.gateway_controller == "on" or (a.gateway_controller == "auto"
                                         and k8s_controller.in_cluster()):
        gw.controller = k8s_controller.GatewayController(a.namespace,
                                                         class_name=a.gateway_class)
    web.run_app(gw.app(), host=a.host, port=a.port, access_log=None)


if __name__ == "__main__":
    main()
