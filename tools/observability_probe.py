"""Run the deployed observability pieces once against real hardware:

1. the GPU exporter (exporter/gpu_exporter.py) on this box's sysfs + `amd-smi`: its
   Prometheus text, plus the raw `amd-smi` JSON it parsed (to pin the schema in fixtures);
2. the kernel-profiler sidecar's window (exporter/kernel_profiler.Profiler.once): an engine
   server is started as a separate CHILD process (this process never touches the GPU), put
   under load over HTTP, and `rocprofv3 --attach <server pid>` collects one kernel-stats window
   of the live engine, rendered as the akap_kernel_* metrics the collector scrapes.

Writes everything under --out (default gpurun_out/obs).

    python tools/observability_probe.py [--out DIR] [--model qwen3-0.6b]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import socket
import subprocess
import sys
import threading
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from aws_k8s_ansible_provisioner_amd.exporter import gpu_exporter, kernel_profiler  # noqa: E402


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def exporter_pass(out: str) -> None:
    raw = {}

    def run(args):  # the exporter passes amd-smi's arguments (it prepends nothing itself)
        args = [shutil.which("amd-smi") or "/opt/rocm/bin/amd-smi", *args]
        r = subprocess.run(args, capture_output=True, text=True, timeout=60)
        raw[" ".join(args)] = {"rc": r.returncode, "stdout": r.stdout[-200000:],
                               "stderr": r.stderr[-4000:]}
        return r.stdout if r.returncode == 0 else None

    exp = gpu_exporter.Exporter("/sys", node=socket.gethostname(), run=run)
    txt = exp.text()
    open(os.path.join(out, "exporter_scrape.txt"), "w").write(txt)
    json.dump(raw, open(os.path.join(out, "amd_smi_raw.json"), "w"), indent=1)
    names = sorted({ln.split("{")[0].split(" ")[0] for ln in txt.splitlines()
                    if ln and not ln.startswith("#")})
    print(f"[exporter] {len(txt.splitlines())} lines, {len(names)} metric names: "
          + ", ".join(names), flush=True)


def profiler_pass(out: str, model: str, window_ms: int) -> None:
    port = _port()
    env = dict(os.environ, PYTHONPATH=ROOT)
    log = open(os.path.join(out, "server.log"), "w")
    srv = subprocess.Popen([sys.executable, "-m", "aws_k8s_ansible_provisioner_amd.server",
                            "--model", model, "--port", str(port), "--host", "127.0.0.1",
                            "--max-num-seqs", "64", "--max-model-len", "2048"],
                           env=env, cwd=ROOT, stdout=log, stderr=subprocess.STDOUT)
    url = f"http://127.0.0.1:{port}"
    stop = threading.Event()
    try:
        t0 = time.time()
        while True:
            try:
                urllib.request.urlopen(url + "/health", timeout=2)
                break
            except Exception:
                if srv.poll() is not None or time.time() - t0 > 300:
                    raise RuntimeError("engine server did not come up (see server.log)")
                time.sleep(1)
        print(f"[profiler] engine pid {srv.pid} up in {time.time() - t0:.1f}s", flush=True)

        def load():
            body = json.dumps({"prompt": "profile window " * 40, "max_tokens": 128,
                               "temperature": 0, "ignore_eos": True}).encode()
            while not stop.is_set():
                try:
                    req = urllib.request.Request(url + "/v1/completions", data=body,
                                                 headers={"Content-Type": "application/json"})
                    urllib.request.urlopen(req, timeout=120).read()
                except Exception:
                    time.sleep(0.2)

        workers = [threading.Thread(target=load, daemon=True) for _ in range(32)]
        for w in workers:
            w.start()
        time.sleep(5)
        prof_dir = os.path.join(out, "prof")
        os.makedirs(prof_dir, exist_ok=True)
        cmds = []

        def run(cmd):
            cmds.append(cmd)
            r = subprocess.run(cmd, capture_output=True, text=True,
                               timeout=90 + window_ms / 1000)
            open(os.path.join(out, "rocprof_attach.log"), "a").write(
                " ".join(cmd) + f"\nrc={r.returncode}\n" + r.stdout[-6000:] + r.stderr[-6000:])
            return r.returncode

        p = kernel_profiler.Profiler(prof_dir, window_ms=window_ms, run=run,
                                     find_pid=lambda: srv.pid)
        ok = p.once()
        txt = p.text()
        open(os.path.join(out, "kernel_profiler_scrape.txt"), "w").write(txt)
        files = sorted(os.path.relpath(os.path.join(d, f), prof_dir)
                       for d, _, fs in os.walk(prof_dir) for f in fs)
        print(f"[profiler] window ok={ok} err={p.last_error!r}; files: {files[:20]}", flush=True)
        print("[profiler] scrape head:\n" + "\n".join(txt.splitlines()[:25]), flush=True)
        m = urllib.request.urlopen(url + "/metrics").read().decode()
        open(os.path.join(out, "engine_metrics.txt"), "w").write(m)
    finally:
        stop.set()
        srv.terminate()
        try:
            srv.wait(timeout=30)
        except subprocess.TimeoutExpired:
            srv.kill()
        log.close()


def inprocess_pass(out: str, model: str) -> None:
    """The engine server (a child process) takes its own kernel-stats windows every 5 s while
    it serves HTTP load; its /metrics must carry the akap_kernel_* series."""
    port = _port()
    env = dict(os.environ, PYTHONPATH=ROOT)
    log = open(os.path.join(out, "server_inprocess.log"), "w")
    srv = subprocess.Popen([sys.executable, "-m", "aws_k8s_ansible_provisioner_amd.server",
                            "--model", model, "--port", str(port), "--host", "127.0.0.1",
                            "--max-num-seqs", "64", "--max-model-len", "2048",
                            "--kernel-stats-interval", "5", "--kernel-stats-window-ms", "1000"],
                           env=env, cwd=ROOT, stdout=log, stderr=subprocess.STDOUT)
    url = f"http://127.0.0.1:{port}"
    stop = threading.Event()
    try:
        t0 = time.time()
        while True:
            try:
                urllib.request.urlopen(url + "/health", timeout=2)
                break
            except Exception:
                if srv.poll() is not None or time.time() - t0 > 300:
                    raise RuntimeError("engine server did not come up (see server_inprocess.log)")
                time.sleep(1)
        print(f"[inprocess] engine up in {time.time() - t0:.1f}s", flush=True)

        def load():
            body = json.dumps({"prompt": "profile window " * 40, "max_tokens": 128,
                               "temperature": 0, "ignore_eos": True}).encode()
            while not stop.is_set():
                try:
                    req = urllib.request.Request(url + "/v1/completions", data=body,
                                                 headers={"Content-Type": "application/json"})
                    urllib.request.urlopen(req, timeout=120).read()
                except Exception:
                    time.sleep(0.2)

        for _ in range(32):
            threading.Thread(target=load, daemon=True).start()
        m = ""
        for _ in range(30):  # a window every 5 s; wait for two
            time.sleep(2)
            m = urllib.request.urlopen(url + "/metrics").read().decode()
            if 'akap_kernel_profiler_windows_total{result="ok"} 2' in m:
                break
        open(os.path.join(out, "engine_metrics_inprocess.txt"), "w").write(m)
        ks = [ln for ln in m.splitlines() if ln.startswith("akap_kernel")]
        print(f"[inprocess] {len(ks)} akap_kernel_* lines; head:\n" + "\n".join(ks[:14]),
              flush=True)
    finally:
        stop.set()
        srv.terminate()
        try:
            srv.wait(timeout=30)
        except subprocess.TimeoutExpired:
            srv.kill()
        log.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "obs"))
    ap.add_argument("--model", default="qwen3-0.6b")
    ap.add_argument("--window-ms", type=int, default=1500)
    ap.add_argument("--skip-profiler", action="store_true")
    ap.add_argument("--inprocess", action="store_true",
                    help="start the server with --kernel-stats-interval (its own torch.profiler "
                         "windows) and scrape its /metrics instead of attaching rocprofv3")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    exporter_pass(a.out)
    if a.inprocess:
        inprocess_pass(a.out, a.model)
    elif not a.skip_profiler:
        profiler_pass(a.out, a.model, a.window_ms)


if __name__ == "__main__":
    main()
