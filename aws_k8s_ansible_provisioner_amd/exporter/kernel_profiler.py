"""Kernel-profiler sidecar: periodic rocprofv3 kernel-stats windows of the LIVE engine,
served as Prometheus metrics for the OTel collector's `akap-kernel-stats` job.

rocprofv3 writes its `--stats` CSVs only when the profiled process exits, so wrapping a
long-running server (`rocprofv3 ... -- python -m ...server`) would never publish anything.
Instead this sidecar (same pod, `shareProcessNamespace: true`, CAP_SYS_PTRACE) attaches to
the running engine for a short window every `--interval` seconds:

    rocprofv3 --attach <engine pid> --attach-duration-msec <window> \\
              --kernel-trace --stats --output-format csv -d <prof>/<n> -o win

keeps the newest `--keep` windows, and serves (rocprof_bridge.render_windows)
  akap_kernel_time_seconds_total / akap_kernel_calls_total   summed over kept windows
  akap_kernel_window_time_fraction{kernel}                    share of GPU kernel time in
                                                              the newest window
  akap_kernel_window_busy_ratio                               kernel time / window length
so per-kernel hot spots (paged attention, decode GEMMs, norms) sit next to the vLLM-style
serving metrics and the GPU exporter's series (SURVEY §5 tracing/profiling, reference
otel-observability-setup.yaml:393-468 scrape jobs).

    python -m aws_k8s_ansible_provisioner_amd.exporter.kernel_profiler --port 9401
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Optional

from . import rocprof_bridge

ENGINE_MARK = "aws_k8s_ansible_provisioner_amd.server"


def find_engine_pid(proc: str = "/proc", mark: str = ENGINE_MARK) -> Optional[int]:
    """PID of the engine process in the shared PID namespace (the python process whose
    command line runs the server module; torchrun's workers for TP: the lowest PID)."""
    found = []
    for d in glob.glob(os.path.join(proc, "[0-9]*")):
        try:
            with open(os.path.join(d, "cmdline"), "rb") as f:
                cmd = f.read().replace(b"\0", b" ").decode(errors="replace")
        except OSError:
            continue
        if mark in cmd and "kernel_profiler" not in cmd and "torchrun" not in cmd.split()[0]:
            found.append(int(os.path.basename(d)))
    return min(found) if found else None


def rocprof_cmd(pid: int, out_dir: str, window_ms: int, exe: str = "rocprofv3") -> list[str]:
    return [exe, "--attach", str(pid), "--attach-duration-msec", str(window_ms),
            "--kernel-trace", "--stats", "--output-format", "csv", "-d", out_dir, "-o", "win"]


class Profiler:
    def __init__(self, prof_dir: str, window_ms: int = 2000, keep: int = 8,
                 run: Optional[Callable[[list[str]], int]] = None,
                 find_pid: Callable[[], Optional[int]] = find_engine_pid):
        self.dir = prof_dir
        self.window_ms = window_ms
        self.keep = keep
        self.run = run or self._run
        self.find_pid = find_pid
        self.n = 0
        self.last_error = ""
        self.failures = 0
        self.ok = 0
        self.last_ok = False

    def _run(self, cmd: list[str]) -> int:
        exe = shutil.which(cmd[0]) or os.path.join("/opt/rocm/bin", cmd[0])
        # the attach needs no input; bounded so a wedged profiler cannot stall the loop
        r = subprocess.run([exe, *cmd[1:]], stdin=subprocess.DEVNULL, capture_output=True,
                           text=True, timeout=60 + cmd_window_s(cmd))
        if r.returncode != 0:
            # e.g. "ptrace call failed. errno: 1 - Operation not permitted": the sidecar needs
            # CAP_SYS_PTRACE and the engine's PID namespace (shareProcessNamespace)
            err = [ln for ln in (r.stderr or "").splitlines() if "failed" in ln.lower()]
            self.last_error = (err[0] if err else (r.stderr or "").strip()[-200:])[-300:]
        return r.returncode

    def windows(self) -> list[str]:
        ws = [d for d in glob.glob(os.path.join(self.dir, "w[0-9]*")) if os.path.isdir(d)]
        return sorted(ws, key=lambda d: int(os.path.basename(d)[1:]))

    def once(self) -> bool:
        pid = self.find_pid()
        if pid is None:
            self.last_error = "engine process not found"
            return False
        out = os.path.join(self.dir, f"w{self.n}")
        self.n += 1
        try:
            rc = self.run(rocprof_cmd(pid, out, self.window_ms))
        except (subprocess.SubprocessError, OSError) as e:
            rc, self.last_error = -1, str(e)
        for old in self.windows()[:-self.keep]:
            shutil.rmtree(old, ignore_errors=True)
        if rc != 0:
            self.last_error = self.last_error or f"rocprofv3 exited {rc}"
            self.failures += 1
            self.last_ok = False
            return False
        self.last_error = ""
        self.ok += 1
        self.last_ok = True
        return True

    def text(self) -> str:
        """The kept windows' akap_kernel_* series plus the sidecar's own health: whether the
        newest window worked, and how many failed (an attach the node forbids shows up here
        instead of as silently empty kernel series)."""
        return rocprof_bridge.render_windows(self.windows(), self.window_ms / 1000.0) + (
            "# HELP akap_kernel_profiler_up 1 if the newest profiling window succeeded\n"
            "# TYPE akap_kernel_profiler_up gauge\n"
            f"akap_kernel_profiler_up {1 if self.last_ok else 0}\n"
            "# HELP akap_kernel_profiler_windows_total Profiling windows attempted, by result\n"
            "# TYPE akap_kernel_profiler_windows_total counter\n"
            f'akap_kernel_profiler_windows_total{{result="ok"}} {self.ok}\n'
            f'akap_kernel_profiler_windows_total{{result="failed"}} {self.failures}\n')


def cmd_window_s(cmd: list[str]) -> float:
    try:
        return int(cmd[cmd.index("--attach-duration-msec") + 1]) / 1000.0
    except (ValueError, IndexError):
        return 0.0


def serve(prof: Profiler, host: str, port: int) -> ThreadingHTTPServer:
    class H(BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            if self.path.startswith("/health"):
                body = b"ok"
            else:
                body = prof.text().encode()
            self.send_response(200)
            self.send_header("Content-Type", "text/plain; version=0.0.4")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    srv = ThreadingHTTPServer((host, port), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def main(argv=None) -> None:
    ap = argparse.ArgumentParser("akap-kernel-profiler")
    ap.add_argument("--dir", default="/prof")
    ap.add_argument("--port", type=int, default=9401)
    ap.add_argument("--interval", type=float, default=120.0, help="seconds between windows")
    ap.add_argument("--window-ms", type=int, default=2000)
    ap.add_argument("--keep", type=int, default=8)
    ap.add_argument("--startup-delay", type=float, default=300.0,
                    help="let the engine load weights / capture graphs first")
    a = ap.parse_args(argv)
    os.makedirs(a.dir, exist_ok=True)
    prof = Profiler(a.dir, a.window_ms, a.keep)
    serve(prof, "0.0.0.0", a.port)
    time.sleep(a.startup_delay)
    while True:
        ok = prof.once()
        if not ok:
            print(f"[kernel-profiler] window skipped: {prof.last_error}", flush=True)
        time.sleep(a.interval)


if __name__ == "__main__":
    main()
