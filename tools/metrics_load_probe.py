"""The engine's own /metrics under load on real hardware: GPU hardware counters
(libakap_pmc.so via ROCP_TOOL_LIBRARIES, --pmc-interval) and in-process kernel-stats windows
(--kernel-stats-interval), scraped while completions stream.

An OpenAI server runs as a CHILD process (this process never touches the GPU); 64 concurrent
/v1/completions requests keep it busy; /metrics is scraped twice during the load.  The
akap_gpu_pmc_* / akap_kernel_* / vllm:* lines are written to --out.

    python tools/metrics_load_probe.py [--out gpurun_out/metrics] [--model qwen3-0.6b]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _get(url: str, timeout: float = 10.0) -> str:
    with urllib.request.urlopen(url, timeout=timeout) as r:
        return r.read().decode()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/metrics")
    ap.add_argument("--model", default="qwen3-0.6b")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    port = _port()
    env = dict(os.environ, ROCP_TOOL_LIBRARIES=os.path.join(
        ROOT, "aws_k8s_ansible_provisioner_amd", "libakap_pmc.so"))
    log = open(os.path.join(a.out, "server.log"), "w")
    srv = subprocess.Popen([sys.executable, "-u", "-m", "aws_k8s_ansible_provisioner_amd.server",
                            "--model", a.model, "--port", str(port), "--pmc-interval", "2",
                            "--kernel-stats-interval", "4", "--max-model-len", "2048"],
                           cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT)
    base = f"http://127.0.0.1:{port}"
    try:
        t0 = time.time()
        while True:
            if srv.poll() is not None:
                raise RuntimeError(f"server exited rc={srv.returncode}")
            try:
                _get(base + "/v1/models", 2.0)
                break
            except OSError:
                if time.time() - t0 > 240:
                    raise RuntimeError("server did not come up")
                time.sleep(1.0)
        print(f"server up in {time.time() - t0:.1f}s", flush=True)
        stop = threading.Event()
        done = [0]

        def client(i):
            body = json.dumps({"prompt": [int(x) for x in range(10 + i, 522 + i)],
                               "max_tokens": 256, "ignore_eos": True}).encode()
            while not stop.is_set():
                req = urllib.request.Request(base + "/v1/completions", data=body,
                                             headers={"Content-Type": "application/json"})
                try:
                    urllib.request.urlopen(req, timeout=120).read()
                    done[0] += 1
                except OSError:
                    time.sleep(0.5)

        th = [threading.Thread(target=client, args=(i,), daemon=True) for i in range(64)]
        for t in th:
            t.start()
        scrapes = []
        for k in range(2):
            time.sleep(10.0)
            text = _get(base + "/metrics")
            keep = [ln for ln in text.splitlines()
                    if ln.startswith(("akap_gpu_pmc", "akap_kernel", "vllm:num_requests",
                                      "vllm:gpu_cache_usage", "vllm:generation_tokens_total"))]
            scrapes.append(keep)
            print(f"scrape {k}: {len(keep)} lines, {done[0]} requests done", flush=True)
        stop.set()
        with open(os.path.join(a.out, "metrics_under_load.prom"), "w") as f:
            for k, keep in enumerate(scrapes):
                f.write(f"# ---- scrape {k} ----\n" + "\n".join(keep) + "\n")
        pmc = [ln for ln in scrapes[-1] if ln.startswith("akap_gpu_pmc")]
        print("\n".join(pmc[:40]), flush=True)
        up = any(ln.startswith("akap_gpu_pmc_up") and ln.rstrip().endswith(" 1") for ln in pmc)
        return 0 if up else 1
    finally:
        srv.terminate()
        try:
            srv.wait(timeout=30)
        except subprocess.TimeoutExpired:
            srv.kill()


if __name__ == "__main__":
    sys.exit(main())
