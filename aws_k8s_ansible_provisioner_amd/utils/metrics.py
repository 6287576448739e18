"""Minimal Prometheus text-format metrics registry (thread-safe, dependency-free).

The engine exports vLLM-style ``vllm:*`` series (what llm-d's endpoint picker and
dashboards read) and, for compatibility with the reference's OTel verification
queries (otel-observability-setup.yaml:727-732, :759-761), the aliases
``vllm_request_total``, ``vllm_active_requests`` and ``vllm_request_duration_seconds``.
"""
from __future__ import annotations

import bisect
import threading
from typing import Iterable, Optional


def _fmt_labels(labels: dict) -> str:
    if not labels:
        return ""
    parts = []
    for k, v in sorted(labels.items()):
        v = str(v).replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')
        parts.append(f'{k}="{v}"')
    return "{" + ",".join(parts) + "}"


class _Metric:
    kind = "untyped"

    def __init__(self, name: str, doc: str, labelnames: Iterable[str] = ()):
        self.name, self.doc = name, doc
        self.labelnames = tuple(labelnames)
        self._lock = threading.Lock()

    def _key(self, labels: dict) -> tuple:
        return tuple(str(labels.get(k, "")) for k in self.labelnames)

    def header(self) -> list[str]:
        return [f"# HELP {self.name} {self.doc}", f"# TYPE {self.name} {self.kind}"]


class Counter(_Metric):
    kind = "counter"

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._v: dict = {}

    def inc(self, amount: float = 1.0, **labels) -> None:
        with self._lock:
            key = self._key(labels)
            self._v[key] = self._v.get(key, 0.0) + amount

    def set_total(self, value: float, **labels) -> None:
        """Mirror a monotonic total kept elsewhere (e.g. the C++ block manager's counts)."""
        with self._lock:
            self._v[self._key(labels)] = float(value)

    def value(self, **labels) -> float:
        return self._v.get(self._key(labels), 0.0)

    def render(self) -> list[str]:
        out = self.header()
        with self._lock:
            items = list(self._v.items()) or ([((), 0.0)] if not self.labelnames else [])
        for key, v in items:
            out.append(f"{self.name}{_fmt_labels(dict(zip(self.labelnames, key)))} {v}")
        return out


class Gauge(_Metric):
    kind = "gauge"

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._v: dict = {}

    def set(self, v: float, **labels) -> None:
        with self._lock:
            self._v[self._key(labels)] = float(v)

    def value(self, **labels) -> float:
        return self._v.get(self._key(labels), 0.0)

    def render(self) -> list[str]:
        out = self.header()
        with self._lock:
            items = list(self._v.items()) or ([((), 0.0)] if not self.labelnames else [])
        for key, v in items:
            out.append(f"{self.name}{_fmt_labels(dict(zip(self.labelnames, key)))} {v}")
        return out


class Histogram(_Metric):
    kind = "histogram"

    def __init__(self, name, doc, buckets: Iterable[float], labelnames=()):
        super().__init__(name, doc, labelnames)
        self.buckets = sorted(buckets)
        self._v: dict = {}

    def observe(self, x: float, **labels) -> None:
        with self._lock:
            key = self._key(labels)
            st = self._v.get(key)
            if st is None:
                st = self._v[key] = [[0] * (len(self.buckets) + 1), 0.0, 0]
            st[0][bisect.bisect_left(self.buckets, x)] += 1
            st[1] += x
            st[2] += 1

    def count(self, **labels) -> int:
        st = self._v.get(self._key(labels))
        return st[2] if st else 0

    def render(self) -> list[str]:
        out = self.header()
        with self._lock:
            items = list(self._v.items())
        for key, (counts, s, n) in items:
            base = dict(zip(self.labelnames, key))
            acc = 0
            for b, c in zip(self.buckets, counts):
                acc += c
                out.append(f"{self.name}_bucket{_fmt_labels({**base, 'le': repr(float(b))})} {acc}")
            out.append(f"{self.name}_bucket{_fmt_labels({**base, 'le': '+Inf'})} {n}")
            out.append(f"{self.name}_sum{_fmt_labels(base)} {s}")
            out.append(f"{self.name}_count{_fmt_labels(base)} {n}")
        return out


class Registry:
    def __init__(self):
        self._m: list[_Metric] = []

    def add(self, m: _Metric) -> _Metric:
        self._m.append(m)
        return m

    def render(self) -> str:
        lines: list[str] = []
        for m in self._m:
            lines.extend(m.render())
        return "\n".join(lines) + "\n"


LAT_BUCKETS = [0.001, 0.005, 0.01, 0.02, 0.04, 0.06, 0.08, 0.1, 0.25, 0.5, 0.75, 1.0, 2.5, 5.0,
               7.5, 10.0, 20.0, 40.0, 80.0]


class EngineMetrics:
    """The serving metric set, labelled by model_name."""

    def __init__(self, model_name: str, registry: Optional[Registry] = None):
        self.model = model_name
        r = self.registry = registry or Registry()
        L = ("model_name",)
        self.running = r.add(Gauge("vllm:num_requests_running", "Requests in the running batch", L))
        self.waiting = r.add(Gauge("vllm:num_requests_waiting", "Requests waiting to be scheduled", L))
        self.kv_usage = r.add(Gauge("vllm:gpu_cache_usage_perc", "Fraction of KV blocks in use", L))
        self.prompt_tokens = r.add(Counter("vllm:prompt_tokens_total", "Prefill tokens processed", L))
        self.gen_tokens = r.add(Counter("vllm:generation_tokens_total", "Generated tokens", L))
        self.success = r.add(Counter("vllm:request_success_total", "Finished requests",
                                     ("model_name", "finished_reason")))
        self.preempt = r.add(Counter("vllm:num_preemptions_total", "Preemptions", L))
        self.prefix_hits = r.add(Counter("vllm:prefix_cache_hits_total", "Prefix-cache hit tokens", L))
        self.prefix_queries = r.add(Counter("vllm:prefix_cache_queries_total", "Prefix-cache queried tokens", L))
        self.ttft = r.add(Histogram("vllm:time_to_first_token_seconds", "TTFT", LAT_BUCKETS, L))
        self.tpot = r.add(Histogram("vllm:time_per_output_token_seconds", "Inter-token latency",
                                    LAT_BUCKETS, L))
        self.e2e = r.add(Histogram("vllm:e2e_request_latency_seconds", "End-to-end latency",
                                   LAT_BUCKETS, L))
        self.queue = r.add(Histogram("vllm:request_queue_time_seconds", "Time waiting before first schedule",
                                     LAT_BUCKETS, L))
        self.step_time = r.add(Histogram("akap:engine_step_seconds", "Engine step wall time",
                                         LAT_BUCKETS, ("model_name", "phase")))
        # disaggregated P/D KV hand-off
        self.kv_held = r.add(Gauge("akap:kv_held_transfers",
                                   "Prefill side: requests whose KV is held for a decode pull", L))
        self.kv_held_expired = r.add(Counter("akap:kv_held_expired_total",
                                             "Held KV freed by the TTL (never pulled)", L))
        self.kv_xfer_fail = r.add(Counter("akap:kv_transfer_failures_total",
                                          "KV sends/receives that failed or timed out", L))
        self.kv_broken = r.add(Gauge("akap:kv_channel_broken",
                                     "1 while the KV-transfer channel awaits a rebuild", L))
        self.kv_resets = r.add(Counter("akap:kv_channel_resets_total",
                                       "KV-transfer channel rebuilds (new process group)", L))
        self.kv_xfer_bytes = r.add(Counter("akap:kv_transfer_bytes_total",
                                           "KV bytes moved over the transfer group",
                                           ("model_name", "direction")))
        self.kv_probe_gbps = r.add(Gauge(
            "akap:kv_channel_probe_gbps",
            "Two-pod P/D: GB/s of the probe transfer over a freshly formed KV channel",
            ("model_name", "peer", "transport", "role")))
        self.kv_ipc = r.add(Gauge(
            "akap:kv_transport_ipc",
            "1 when this engine moves KV by the hipIpc pull (no failed peer mapping)", L))
        # aliases queried by the reference's OTel verification play
        self.req_total = r.add(Counter("vllm_request_total", "Requests received (alias)", L))
        self.active = r.add(Gauge("vllm_active_requests", "Requests in flight (alias)", L))
        self.duration = r.add(Histogram("vllm_request_duration_seconds", "Request duration (alias)",
                                        LAT_BUCKETS, L))

    def render(self) -> str:
        return self.registry.render()
