"""rocprofv3 -> Prometheus bridge: exposes per-kernel GPU time from rocprofv3
`--kernel-trace --stats` CSVs (``*_kernel_stats.csv``) found under a directory, so kernel
hot spots (paged attention, GEMMs, norms) are visible in the OTel pipeline next to the
serving and GPU metrics.

    rocprofv3 --kernel-trace --stats -d /prof -o run --output-format csv -- python3 -m ...server
    python -m aws_k8s_ansible_provisioner_amd.exporter.rocprof_bridge --dir /prof --port 9401
(the engine pod annotates akap.rocprof/port so the collector's akap-kernel-stats job finds it)
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


def collect(directory: str) -> dict[str, tuple[float, int]]:
    agg: dict[str, tuple[float, int]] = {}
    for path in glob.glob(os.path.join(directory, "**", "*kernel_stats.csv"), recursive=True):
        try:
            with open(path) as f:
                for r in csv.DictReader(f):
                    name = r["Name"][:160]
                    t, n = agg.get(name, (0.0, 0))
                    agg[name] = (t + float(r["TotalDurationNs"]) * 1e-9, n + int(r["Calls"]))
        except (OSError, KeyError, ValueError):
            continue
    return agg


def render(agg: dict[str, tuple[float, int]]) -> str:
    def esc(s):
        return s.replace("\\", "\\\\").replace('"', '\\"').replace("\n", " ")

    lines = ["# HELP akap_kernel_time_seconds_total GPU time per kernel (rocprofv3 stats)",
             "# TYPE akap_kernel_time_seconds_total counter"]
    for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        lines.append(f'akap_kernel_time_seconds_total{{kernel="{esc(k)}"}} {t}')
    lines += ["# HELP akap_kernel_calls_total Kernel dispatches (rocprofv3 stats)",
              "# TYPE akap_kernel_calls_total counter"]
    for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        lines.append(f'akap_kernel_calls_total{{kernel="{esc(k)}"}} {n}')
    return "\n".join(lines) + "\n"


def render_windows(windows: list[str], window_s: float) -> str:
    """kernel_profiler.py's view: cumulative counters over every kept attach window plus
    the newest window's per-kernel share of GPU kernel time and its busy ratio."""
    return render_aggregates([collect(w) for w in windows], window_s)


def render_aggregates(windows: list[dict], window_s: float) -> str:
    """The same view from per-window {kernel: (seconds, calls)} maps (rocprofv3 CSV windows or
    the in-process torch.profiler windows of exporter/inprocess_profiler.py)."""
    agg: dict[str, tuple[float, int]] = {}
    for w in windows:
        for k, (t, n) in w.items():
            t0, n0 = agg.get(k, (0.0, 0))
            agg[k] = (t0 + t, n0 + n)
    lines = [render(agg).rstrip("\n")]
    last = windows[-1] if windows else {}
    tot = sum(t for t, _ in last.values())

    def esc(s):
        return s.replace("\\", "\\\\").replace('"', '\\"').replace("\n", " ")

    lines += ["# HELP akap_kernel_window_time_fraction Share of GPU kernel time in the newest "
              "profiling window", "# TYPE akap_kernel_window_time_fraction gauge"]
    for k, (t, _) in sorted(last.items(), key=lambda kv: -kv[1][0]):
        lines.append(f'akap_kernel_window_time_fraction{{kernel="{esc(k)}"}} '
                     f'{t / tot if tot else 0.0}')
    lines += ["# HELP akap_kernel_window_busy_ratio GPU kernel time / window length (newest)",
              "# TYPE akap_kernel_window_busy_ratio gauge",
              f"akap_kernel_window_busy_ratio {tot / window_s if window_s and last else 0.0}",
              "# HELP akap_kernel_windows Profiling windows kept",
              "# TYPE akap_kernel_windows gauge", f"akap_kernel_windows {len(windows)}"]
    return "\n".join(lines) + "\n"


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/prof")
    ap.add_argument("--port", type=int, default=9401)
    a = ap.parse_args(argv)

    class H(BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            body = render(collect(a.dir)).encode()
            self.send_response(200)
            self.send_header("Content-Type", "text/plain; version=0.0.4")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *x):
            pass

    ThreadingHTTPServer(("0.0.0.0", a.port), H).serve_forever()


if __name__ == "__main__":
    main()
