"""Request tracing: OTLP/HTTP-JSON span export + W3C trace-context propagation.

SURVEY §5 "Tracing": the reference's OTel collector receives OTLP traces
(`otel-observability-setup.yaml:504-509,633-636`) but nothing emits them.  Here the
engine emits one `llm_request` span per request with `prefill` (arrival -> first token)
and `decode` (first token -> finish) children, and the gateway emits a `gateway.route`
span and forwards `traceparent` so both hops join one trace.

No opentelemetry SDK is required (none is installed in the serving image): spans are
buffered and POSTed by a daemon thread as OTLP/JSON to ``<endpoint>/v1/traces`` (the
collector's :4318 http receiver, deploy/otel/collector.yaml.j2).  Export never blocks the
engine loop: a full buffer or a failed POST drops spans and counts them.

Configuration: ``--otlp-traces-endpoint`` (server / gateway flag, same name as vLLM's) or
the standard ``OTEL_EXPORTER_OTLP_TRACES_ENDPOINT`` / ``OTEL_EXPORTER_OTLP_ENDPOINT``
environment variables; ``OTEL_SERVICE_NAME`` names the service.
"""
from __future__ import annotations

import json
import os
import re
import secrets
import threading
import time
import urllib.request
from typing import Optional

SPAN_KIND_INTERNAL, SPAN_KIND_SERVER, SPAN_KIND_CLIENT = 1, 2, 3
_TRACEPARENT = re.compile(r"^([0-9a-f]{2})-([0-9a-f]{32})-([0-9a-f]{16})-([0-9a-f]{2})$")


def new_trace_id() -> str:
    return secrets.token_hex(16)


def new_span_id() -> str:
    return secrets.token_hex(8)


def parse_traceparent(header: Optional[str]) -> tuple[Optional[str], Optional[str]]:
    """W3C traceparent -> (trace_id, parent_span_id); (None, None) when absent/invalid."""
    if not header:
        return None, None
    m = _TRACEPARENT.match(header.strip().lower())
    if not m or m.group(2) == "0" * 32 or m.group(3) == "0" * 16:
        return None, None
    return m.group(2), m.group(3)


def make_traceparent(trace_id: str, span_id: str) -> str:
    return f"00-{trace_id}-{span_id}-01"


def _attr(k: str, v) -> dict:
    if isinstance(v, bool):
        val = {"boolValue": v}
    elif isinstance(v, int):
        val = {"intValue": str(v)}
    elif isinstance(v, float):
        val = {"doubleValue": v}
    else:
        val = {"stringValue": str(v)}
    return {"key": k, "value": val}


class OTLPTracer:
    def __init__(self, endpoint: str, service_name: str = "akap-engine",
                 flush_interval: float = 1.0, max_buffer: int = 8192, timeout: float = 2.0,
                 resource: Optional[dict] = None):
        ep = endpoint.rstrip("/")
        if not ep.startswith("http"):
            ep = "http://" + ep
        self.url = ep if ep.endswith("/v1/traces") else ep + "/v1/traces"
        self.service_name = service_name
        self.flush_interval = flush_interval
        self.max_buffer = max_buffer
        self.timeout = timeout
        self.resource = dict(resource or {})
        self._buf: list = []
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self._stop = False
        self.exported = 0
        self.dropped = 0
        self._thread = threading.Thread(target=self._run, daemon=True, name="otlp-export")
        self._thread.start()

    # ------------------------------------------------------------------ recording
    def record(self, name: str, start: float, end: float, trace_id: Optional[str] = None,
               parent_span_id: Optional[str] = None, span_id: Optional[str] = None,
               kind: int = SPAN_KIND_INTERNAL, attributes: Optional[dict] = None,
               error: bool = False) -> tuple[str, str]:
        """Record a finished span (times in epoch seconds).  Returns (trace_id, span_id)."""
        trace_id = trace_id or new_trace_id()
        span_id = span_id or new_span_id()
        span = {"traceId": trace_id, "spanId": span_id, "name": name, "kind": kind,
                "startTimeUnixNano": str(int(start * 1e9)),
                "endTimeUnixNano": str(int(max(end, start) * 1e9)),
                "attributes": [_attr(k, v) for k, v in (attributes or {}).items()
                               if v is not None],
                "status": {"code": 2 if error else 1}}
        if parent_span_id:
            span["parentSpanId"] = parent_span_id
        with self._lock:
            if len(self._buf) >= self.max_buffer:
                self.dropped += 1
            else:
                self._buf.append(span)
        return trace_id, span_id

    # ------------------------------------------------------------------ export
    def payload(self, spans: list) -> dict:
        res = {"service.name": self.service_name, **self.resource}
        return {"resourceSpans": [{
            "resource": {"attributes": [_attr(k, v) for k, v in res.items()]},
            "scopeSpans": [{"scope": {"name": "aws_k8s_ansible_provisioner_amd"},
                            "spans": spans}]}]}

    def flush(self) -> int:
        with self._lock:
            spans, self._buf = self._buf, []
        if not spans:
            return 0
        body = json.dumps(self.payload(spans)).encode()
        req = urllib.request.Request(self.url, data=body, method="POST",
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                r.read()
            self.exported += len(spans)
        except Exception:
            self.dropped += len(spans)
        return len(spans)

    def _run(self) -> None:
        while not self._stop:
            self._wake.wait(self.flush_interval)
            self._wake.clear()
            self.flush()

    def shutdown(self) -> None:
        self._stop = True
        self._wake.set()
        self._thread.join(timeout=self.timeout + 1)
        self.flush()


_TRACER: Optional[OTLPTracer] = None


def configure(endpoint: Optional[str] = None, service_name: Optional[str] = None,
              **kw) -> Optional[OTLPTracer]:
    """Install the process-wide tracer (None endpoint + no env var -> tracing off)."""
    global _TRACER
    endpoint = (endpoint or os.environ.get("OTEL_EXPORTER_OTLP_TRACES_ENDPOINT")
                or os.environ.get("OTEL_EXPORTER_OTLP_ENDPOINT"))
    if _TRACER is not None:
        _TRACER.shutdown()
        _TRACER = None
    if endpoint:
        _TRACER = OTLPTracer(endpoint, service_name or os.environ.get("OTEL_SERVICE_NAME",
                                                                      "akap-engine"), **kw)
    return _TRACER


def get_tracer() -> Optional[OTLPTracer]:
    return _TRACER


def record_request(tr: OTLPTracer, *, req_id: str, model: str, arrival: float,
                   first_token: Optional[float], finish: float, prompt_tokens: int,
                   completion_tokens: int, finish_reason: Optional[str], max_tokens: int,
                   temperature: float, top_p: float, traceparent: Optional[str] = None,
                   cached_tokens: int = 0) -> str:
    """Engine-side request span + phase children.  Returns the trace id."""
    trace_id, parent = parse_traceparent(traceparent)
    trace_id = trace_id or new_trace_id()
    root = new_span_id()
    attrs = {"gen_ai.system": "akap", "gen_ai.request.id": req_id,
             "gen_ai.response.model": model, "gen_ai.request.max_tokens": max_tokens,
             "gen_ai.request.temperature": float(temperature),
             "gen_ai.request.top_p": float(top_p),
             "gen_ai.usage.prompt_tokens": prompt_tokens,
             "gen_ai.usage.completion_tokens": completion_tokens,
             "gen_ai.usage.cached_tokens": cached_tokens,
             "gen_ai.response.finish_reason": finish_reason or "",
             "gen_ai.latency.e2e": finish - arrival}
    if first_token is not None:
        attrs["gen_ai.latency.time_to_first_token"] = first_token - arrival
        if completion_tokens > 1:
            attrs["gen_ai.latency.time_per_output_token"] = \
                (finish - first_token) / (completion_tokens - 1)
    tr.record("llm_request", arrival, finish, trace_id, parent, root, SPAN_KIND_SERVER, attrs,
              error=finish_reason == "abort")
    ft = first_token if first_token is not None else finish
    tr.record("prefill", arrival, ft, trace_id, root,
              attributes={"gen_ai.usage.prompt_tokens": prompt_tokens})
    if first_token is not None and finish > first_token:
        tr.record("decode", first_token, finish, trace_id, root,
                  attributes={"gen_ai.usage.completion_tokens": completion_tokens})
    return trace_id


class Span:
    """Context manager for an in-process span (gateway hop, server handler)."""

    def __init__(self, name: str, traceparent: Optional[str] = None,
                 kind: int = SPAN_KIND_SERVER, attributes: Optional[dict] = None):
        self.name = name
        self.trace_id, self.parent = parse_traceparent(traceparent)
        self.trace_id = self.trace_id or new_trace_id()
        self.span_id = new_span_id()
        self.kind = kind
        self.attributes = dict(attributes or {})
        self.error = False

    @property
    def traceparent(self) -> str:
        return make_traceparent(self.trace_id, self.span_id)

    def __enter__(self):
        self.start = time.time()
        return self

    def __exit__(self, et, ev, tb):
        tr = get_tracer()
        if tr is not None:
            tr.record(self.name, self.start, time.time(), self.trace_id, self.parent,
                      self.span_id, self.kind, self.attributes, error=self.error or et is not None)
        return False
