"""MI355X GPU metrics exporter (Prometheus text on :9400, port name `gpu-metrics`).

Replaces the NVIDIA GPU Operator's DCGM exporter the reference scrapes
(kubernetes-single-node.yaml:480-503, otel-observability-setup.yaml:393-468, queried at
:735-743 and :764-767).  Sources, in order: the amdgpu sysfs interface (no tools needed,
works from a DaemonSet with /sys mounted read-only), then `amd-smi metric --json` if the
binary is present.  Every series is exported under amd_gpu_* names and under the
DCGM_FI_DEV_* names the reference's dashboards/queries use.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import shutil
import socket
import subprocess
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Optional

AMD_VENDOR = "0x1002"


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _num(path: str) -> Optional[float]:
    s = _read(path)
    try:
        return float(s) if s is not None else None
    except ValueError:
        return None


def read_sysfs(root: str = "/sys") -> list[dict]:
    gpus = []
    cards = sorted(glob.glob(os.path.join(root, "class", "drm", "card[0-9]*")),
                   key=lambda p: int(os.path.basename(p)[4:]) if os.path.basename(p)[4:].isdigit() else 1 << 30)
    idx = 0
    for card in cards:
        name = os.path.basename(card)
        if not name[4:].isdigit():
            continue
        dev = os.path.join(card, "device")
        if _read(os.path.join(dev, "vendor")) != AMD_VENDOR:
            continue
        g = {"gpu": idx, "card": name,
             "pci": os.path.basename(os.path.realpath(dev)),
             "model": _read(os.path.join(dev, "product_name")) or "AMD Instinct MI355X",
             "util": _num(os.path.join(dev, "gpu_busy_percent")),
             "mem_busy": _num(os.path.join(dev, "mem_busy_percent")),
             "vram_used": _num(os.path.join(dev, "mem_info_vram_used")),
             "vram_total": _num(os.path.join(dev, "mem_info_vram_total")),
             "temps": {}, "power_w": None}
        for hw in glob.glob(os.path.join(dev, "hwmon", "hwmon*")):
            for t in glob.glob(os.path.join(hw, "temp*_input")):
                label = _read(t.replace("_input", "_label")) or os.path.basename(t)[:-6]
                v = _num(t)
                if v is not None:
                    g["temps"][label] = v / 1000.0
            for pname in ("power1_average", "power1_input"):
                v = _num(os.path.join(hw, pname))
                if v is not None:
                    g["power_w"] = v / 1e6
                    break
        gpus.append(g)
        idx += 1
    return gpus


def read_amdsmi() -> list[dict]:
    exe = shutil.which("amd-smi")
    if not exe:
        return []
    try:
        out = subprocess.run([exe, "metric", "--json"], capture_output=True, text=True,
                             timeout=10).stdout
        data = json.loads(out)
    except (subprocess.SubprocessError, ValueError, OSError):
        return []
    gpus = []
    for i, m in enumerate(data if isinstance(data, list) else data.get("gpu_data", [])):
        def val(*keys):
            cur = m
            for k in keys:
                if not isinstance(cur, dict) or k not in cur:
                    return None
                cur = cur[k]
            if isinstance(cur, dict):
                cur = cur.get("value")
            try:
                return float(cur)
            except (TypeError, ValueError):
                return None
        gpus.append({"gpu": m.get("gpu", i), "card": f"gpu{i}", "pci": "", "model": "AMD Instinct",
                     "util": val("usage", "gfx_activity"), "mem_busy": val("usage", "umc_activity"),
                     "vram_used": (val("mem_usage", "used_vram") or 0) * 2**20,
                     "vram_total": (val("mem_usage", "total_vram") or 0) * 2**20,
                     "temps": {k: v for k, v in {"edge": val("temperature", "edge"),
                                                  "junction": val("temperature", "hotspot"),
                                                  "mem": val("temperature", "mem")}.items()
                               if v is not None},
                     "power_w": val("power", "socket_power")})
    return gpus


def render(gpus: list[dict], node: str) -> str:
    L = []

    def emit(name, help_, typ, samples):
        L.append(f"# HELP {name} {help_}")
        L.append(f"# TYPE {name} {typ}")
        for labels, v in samples:
            if v is None:
                continue
            lab = ",".join(f'{k}="{val}"' for k, val in labels.items())
            L.append(f"{name}{{{lab}}} {v}")

    def lbl(g, **extra):
        d = {"gpu": g["gpu"], "pci_bus_id": g["pci"], "modelName": g["model"], "Hostname": node}
        d.update(extra)
        return d

    temp = lambda g: g["temps"].get("junction", g["temps"].get("edge", next(iter(g["temps"].values()), None)))  # noqa: E731
    emit("amd_gpu_utilization_percent", "GFX engine busy %", "gauge", [(lbl(g), g["util"]) for g in gpus])
    emit("amd_gpu_memory_busy_percent", "Memory controller busy %", "gauge", [(lbl(g), g["mem_busy"]) for g in gpus])
    emit("amd_gpu_vram_used_bytes", "VRAM (HBM) used", "gauge", [(lbl(g), g["vram_used"]) for g in gpus])
    emit("amd_gpu_vram_total_bytes", "VRAM (HBM) total", "gauge", [(lbl(g), g["vram_total"]) for g in gpus])
    emit("amd_gpu_temperature_celsius", "Sensor temperature", "gauge",
         [(lbl(g, sensor=k), v) for g in gpus for k, v in g["temps"].items()])
    emit("amd_gpu_power_watts", "Socket power", "gauge", [(lbl(g), g["power_w"]) for g in gpus])
    # DCGM-compatible aliases (names the reference's OTel play and dashboards query)
    emit("DCGM_FI_DEV_GPU_UTIL", "GPU utilization (alias)", "gauge", [(lbl(g), g["util"]) for g in gpus])
    emit("DCGM_FI_DEV_MEM_COPY_UTIL", "Memory utilization (alias)", "gauge", [(lbl(g), g["mem_busy"]) for g in gpus])
    emit("DCGM_FI_DEV_GPU_TEMP", "GPU temperature C (alias)", "gauge", [(lbl(g), temp(g)) for g in gpus])
    emit("DCGM_FI_DEV_POWER_USAGE", "Power W (alias)", "gauge", [(lbl(g), g["power_w"]) for g in gpus])
    emit("DCGM_FI_DEV_FB_USED", "Framebuffer used MiB (alias)", "gauge",
         [(lbl(g), None if g["vram_used"] is None else g["vram_used"] / 2**20) for g in gpus])
    emit("DCGM_FI_DEV_FB_FREE", "Framebuffer free MiB (alias)", "gauge",
         [(lbl(g), None if g["vram_used"] is None or g["vram_total"] is None
           else (g["vram_total"] - g["vram_used"]) / 2**20) for g in gpus])
    emit("amd_gpu_exporter_gpus", "GPUs found", "gauge", [({"Hostname": node}, len(gpus))])
    return "\n".join(L) + "\n"


class Exporter:
    def __init__(self, sysfs_root: str = "/sys", node: Optional[str] = None, ttl: float = 1.0):
        self.root = sysfs_root
        self.node = node or os.environ.get("NODE_NAME") or socket.gethostname()
        self.ttl = ttl
        self._cache = (0.0, "")
        self._lock = threading.Lock()

    def collect(self) -> list[dict]:
        return read_sysfs(self.root) or read_amdsmi()

    def text(self) -> str:
        with self._lock:
            t, txt = self._cache
            if time.time() - t > self.ttl:
                txt = render(self.collect(), self.node)
                self._cache = (time.time(), txt)
            return txt


def serve(exp: Exporter, host: str, port: int) -> ThreadingHTTPServer:
    class H(BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            if self.path.startswith("/metrics"):
                body = exp.text().encode()
                self.send_response(200)
                self.send_header("Content-Type", "text/plain; version=0.0.4")
            elif self.path.startswith("/health"):
                body = b"ok"
                self.send_response(200)
                self.send_header("Content-Type", "text/plain")
            else:
                body = b"not found"
                self.send_response(404)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    srv = ThreadingHTTPServer((host, port), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def main(argv=None) -> None:
    ap = argparse.ArgumentParser("akap-gpu-exporter")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=9400)
    ap.add_argument("--sysfs-root", default="/sys")
    a = ap.parse_args(argv)
    serve(Exporter(a.sysfs_root), a.host, a.port)
    while True:
        time.sleep(3600)


if __name__ == "__main__":
    main()
