"""MI355X GPU metrics exporter (Prometheus text on :9400, port name `gpu-metrics`).

Replaces the NVIDIA GPU Operator's DCGM exporter the reference scrapes
(kubernetes-single-node.yaml:480-503, otel-observability-setup.yaml:393-468, queried at
:735-743 and :764-767).  Sources, in order: the amdgpu sysfs interface (no tools needed,
works from a DaemonSet with /sys mounted read-only), then `amd-smi metric --json` if the
binary is present.  Every series is exported under amd_gpu_* names and under the
DCGM_FI_DEV_* names the reference's dashboards/queries use.

Beyond utilisation / memory / temperature / power (the DCGM defaults the reference's
ServiceMonitor collects), the exporter reads what an 8-GPU xGMI node needs watched:
  * clocks       sysfs pp_dpm_{sclk,mclk,fclk,socclk} current level (or amd-smi `clock`)
  * ECC / RAS    sysfs ras/<block>_err_count (ue / ce) (or amd-smi `ecc` / `ecc_blocks`)
  * PCIe replays sysfs pcie_replay_count, energy: hwmon energy1_input
  * xGMI         `amd-smi xgmi -m --json`: per-peer-link read / write data (KB counters),
                 link bit rate and max bandwidth; `amd-smi metric` xgmi_err status
The amd-smi JSON shapes follow /opt/rocm/libexec/amdsmi_cli (ROCm 7.2) amdsmi_commands.py
(metric: values_dict['clock'|'ecc'|'ecc_blocks'|'pcie'|'energy'|'xgmi_err'];
xgmi -m: [{gpu, bdf, link_metrics: {bit_rate, max_bandwidth, link_type, links: [{gpu, bdf,
read, write}]}}], optionally under {"xgmi_metric": [...]}).
"""
from __future__ import annotations

import argparse
import glob
import json
import re
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
        g["clocks"] = _dpm_clocks(dev)
        g["ecc"] = _ras_counts(dev)
        g["pcie_replay"] = _num(os.path.join(dev, "pcie_replay_count"))
        for hw in glob.glob(os.path.join(dev, "hwmon", "hwmon*")):
            v = _num(os.path.join(hw, "energy1_input"))  # microjoules
            if v is not None:
                g["energy_j"] = v / 1e6
        gpus.append(g)
        idx += 1
    return gpus


_DPM = {"gfx": "pp_dpm_sclk", "mem": "pp_dpm_mclk", "fabric": "pp_dpm_fclk", "soc": "pp_dpm_socclk"}


def _dpm_clocks(dev: str) -> dict:
    """Current DPM level of each clock domain: the line marked '*' ("1: 2100Mhz *")."""
    out = {}
    for dom, fname in _DPM.items():
        txt = _read(os.path.join(dev, fname))
        if not txt:
            continue
        for line in txt.splitlines():
            if line.rstrip().endswith("*"):
                tok = line.split(":", 1)[-1].strip().split()[0].lower()
                try:
                    out[dom] = float(tok.replace("mhz", ""))
                except ValueError:
                    pass
                break
    return out


def _ras_counts(dev: str) -> dict:
    """sysfs RAS error counters: ras/<block>_err_count holds "ue: N" / "ce: N" (/ "de: N")
    lines -> {block: {"uncorrectable": N, "correctable": N[, "deferred": N]}}."""
    out = {}
    kinds = {"ue": "uncorrectable", "ce": "correctable", "de": "deferred"}
    for path in glob.glob(os.path.join(dev, "ras", "*_err_count")):
        block = os.path.basename(path)[: -len("_err_count")]
        txt = _read(path) or ""
        d = {}
        for line in txt.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in kinds:
                try:
                    d[kinds[k.strip()]] = float(v.strip())
                except ValueError:
                    pass
        if d:
            out[block] = d
    return out


_BUS = re.compile(r"^[0-9a-f]{4}:[0-9a-f]{2}:[0-9a-f]{2}\.[0-7]$")


def _run_amdsmi(args: list[str]) -> Optional[str]:
    exe = shutil.which("amd-smi")
    if not exe:
        return None
    try:
        return subprocess.run([exe, *args], capture_output=True, text=True, timeout=10).stdout
    except (subprocess.SubprocessError, OSError):
        return None


def _v(x) -> Optional[float]:
    """amd-smi JSON scalar: a number, {"value": n, "unit": u}, or "N/A"."""
    if isinstance(x, dict):
        x = x.get("value")
    try:
        return float(x)
    except (TypeError, ValueError):
        return None


def read_amdsmi_bdf(run=_run_amdsmi) -> dict:
    """`amd-smi list --json` -> {amd-smi gpu index: PCI bus id}.  amd-smi numbers only the GPUs
    visible to this process (a container granted one GPU sees "gpu 0" while sysfs lists the
    node's eight cards), so its per-GPU data is matched to sysfs cards by bus id, never by
    index (seen on an MI355X box: amd-smi gpu 0 = sysfs card 2, 0000:5d:00.0)."""
    out = run(["list", "--json"])
    if not out:
        return {}
    try:
        data = json.loads(out)
    except ValueError:
        return {}
    if isinstance(data, dict):
        data = data.get("gpu_list") or data.get("gpus") or list(data.values())
    res = {}
    for e in data if isinstance(data, list) else []:
        if isinstance(e, dict) and "gpu" in e and isinstance(e.get("bdf"), str):
            res[e["gpu"]] = e["bdf"].lower()
    return res


def read_amdsmi(run=_run_amdsmi) -> list[dict]:
    bdf = read_amdsmi_bdf(run)
    out = run(["metric", "--json"])
    if not out:
        return []
    try:
        data = json.loads(out)
    except ValueError:
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
        gpus.append({"gpu": m.get("gpu", i), "card": f"gpu{i}", "pci": bdf.get(m.get("gpu", i), ""),
                     "model": "AMD Instinct",
                     "util": val("usage", "gfx_activity"), "mem_busy": val("usage", "umc_activity"),
                     "vram_used": (val("mem_usage", "used_vram") or 0) * 2**20,
                     "vram_total": (val("mem_usage", "total_vram") or 0) * 2**20,
                     "temps": {k: v for k, v in {"edge": val("temperature", "edge"),
                                                  "junction": val("temperature", "hotspot"),
                                                  "mem": val("temperature", "mem")}.items()
                               if v is not None},
                     "power_w": val("power", "socket_power"),
                     **_amdsmi_extras(m)})
    return gpus


_SMI_CLK = {"gfx_0": "gfx", "mem_0": "mem", "fclk_0": "fabric", "socclk_0": "soc"}


def _amdsmi_extras(m: dict) -> dict:
    """clocks / ECC / PCIe replay / energy / xGMI error status of one `amd-smi metric` GPU."""
    ex: dict = {"clocks": {}, "ecc": {}}
    clk = m.get("clock")
    if isinstance(clk, dict):
        for key, dom in _SMI_CLK.items():
            c = clk.get(key)
            v = _v(c.get("clk")) if isinstance(c, dict) else None
            if v is not None:
                ex["clocks"][dom] = v
    blocks = m.get("ecc_blocks")
    if isinstance(blocks, dict):
        for b, d in blocks.items():
            if isinstance(d, dict):
                e = {k: _v(d.get(f"{k}_count")) for k in ("correctable", "uncorrectable",
                                                         "deferred")}
                e = {k: v for k, v in e.items() if v is not None}
                if e:
                    ex["ecc"][b.lower()] = e
    ecc = m.get("ecc")
    if not ex["ecc"] and isinstance(ecc, dict):
        e = {k: _v(ecc.get(f"total_{k}_count")) for k in ("correctable", "uncorrectable",
                                                          "deferred")}
        e = {k: v for k, v in e.items() if v is not None}
        if e:
            ex["ecc"]["total"] = e
    pcie = m.get("pcie")
    if isinstance(pcie, dict):
        ex["pcie_replay"] = _v(pcie.get("replay_count"))
    en = m.get("energy")
    if isinstance(en, dict):
        e = en.get("total_energy_consumption")
        v = _v(e)
        unit = e.get("unit", "J") if isinstance(e, dict) else "J"
        if v is not None:
            ex["energy_j"] = v / 1e6 if unit.lower() in ("uj", "µj") else v
    xe = m.get("xgmi_err")
    if isinstance(xe, str) and xe != "N/A":
        ex["xgmi_err"] = 0.0 if "NO_ERR" in xe.upper() else 1.0
    return ex


def read_xgmi(run=_run_amdsmi) -> dict:
    """`amd-smi xgmi -m --json` -> {gpu: {"bit_rate": Gb/s, "max_bw": Gb/s, "links":
    {peer_gpu: (read_bytes, write_bytes)}}} (the CLI reports cumulative KB per peer)."""
    out = run(["xgmi", "-m", "--json"])
    if not out:
        return {}
    try:
        data = json.loads(out)
    except ValueError:
        return {}
    if isinstance(data, dict):
        data = data.get("xgmi_metric", [])

    def flat(x):
        if isinstance(x, list):
            for y in x:
                yield from flat(y)
        elif isinstance(x, dict):
            yield x

    res = {}
    for d in flat(data):
        lm = d.get("link_metrics")
        if not isinstance(lm, dict) or "gpu" not in d:
            continue
        links = {}
        for ln in lm.get("links", []) or []:
            if not isinstance(ln, dict) or ln.get("gpu") == d["gpu"]:
                continue
            r, w = _v(ln.get("read")), _v(ln.get("write"))
            if r is None and w is None:
                continue
            links[ln.get("gpu")] = (None if r is None else r * 1024,
                                    None if w is None else w * 1024)
        res[d["gpu"]] = {"bit_rate": _v(lm.get("bit_rate")),
                         "max_bw": _v(lm.get("max_bandwidth")), "links": links,
                         "pci": str(d.get("bdf", "")).lower()}
    return res


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
    clocks = [(g, dom, v) for g in gpus for dom, v in (g.get("clocks") or {}).items()]
    emit("amd_gpu_clock_mhz", "Current DPM clock per domain", "gauge",
         [(lbl(g, domain=dom), v) for g, dom, v in clocks])
    emit("DCGM_FI_DEV_SM_CLOCK", "GFX clock MHz (alias)", "gauge",
         [(lbl(g), v) for g, dom, v in clocks if dom == "gfx"])
    emit("DCGM_FI_DEV_MEM_CLOCK", "Memory clock MHz (alias)", "gauge",
         [(lbl(g), v) for g, dom, v in clocks if dom == "mem"])
    ecc = [(g, b, k, v) for g in gpus for b, d in (g.get("ecc") or {}).items()
           for k, v in d.items()]
    emit("amd_gpu_ecc_errors_total", "RAS error count per block and kind", "counter",
         [(lbl(g, block=b, kind=k), v) for g, b, k, v in ecc])

    def ecc_sum(g, kind):
        vals = [d.get(kind) for d in (g.get("ecc") or {}).values() if d.get(kind) is not None]
        return sum(vals) if vals else None
    emit("DCGM_FI_DEV_ECC_SBE_VOL_TOTAL", "Correctable ECC errors (alias)", "counter",
         [(lbl(g), ecc_sum(g, "correctable")) for g in gpus])
    emit("DCGM_FI_DEV_ECC_DBE_VOL_TOTAL", "Uncorrectable ECC errors (alias)", "counter",
         [(lbl(g), ecc_sum(g, "uncorrectable")) for g in gpus])
    emit("amd_gpu_pcie_replay_total", "PCIe replay count", "counter",
         [(lbl(g), g.get("pcie_replay")) for g in gpus])
    emit("DCGM_FI_DEV_PCIE_REPLAY_COUNTER", "PCIe replays (alias)", "counter",
         [(lbl(g), g.get("pcie_replay")) for g in gpus])
    emit("amd_gpu_energy_joules_total", "Energy consumed", "counter",
         [(lbl(g), g.get("energy_j")) for g in gpus])
    emit("DCGM_FI_DEV_TOTAL_ENERGY_CONSUMPTION", "Energy mJ (alias)", "counter",
         [(lbl(g), None if g.get("energy_j") is None else g["energy_j"] * 1e3) for g in gpus])
    emit("amd_gpu_xgmi_error", "xGMI error status (0 = no error)", "gauge",
         [(lbl(g), g.get("xgmi_err")) for g in gpus])
    xl = [(g, peer, rw) for g in gpus for peer, rw in ((g.get("xgmi") or {}).get("links") or {}).items()]
    emit("amd_gpu_xgmi_read_bytes_total", "xGMI data read from a peer GPU", "counter",
         [(lbl(g, peer_gpu=p), rw[0]) for g, p, rw in xl])
    emit("amd_gpu_xgmi_write_bytes_total", "xGMI data written to a peer GPU", "counter",
         [(lbl(g, peer_gpu=p), rw[1]) for g, p, rw in xl])
    emit("amd_gpu_xgmi_link_bitrate_gbps", "xGMI link bit rate", "gauge",
         [(lbl(g), (g.get("xgmi") or {}).get("bit_rate")) for g in gpus])
    emit("amd_gpu_xgmi_max_bandwidth_gbps", "xGMI link max bandwidth", "gauge",
         [(lbl(g), (g.get("xgmi") or {}).get("max_bw")) for g in gpus])

    def xsum(g, i):
        vals = [rw[i] for rw in ((g.get("xgmi") or {}).get("links") or {}).values()
                if rw[i] is not None]
        return sum(vals) if vals else None
    emit("DCGM_FI_PROF_NVLINK_RX_BYTES", "xGMI bytes read, all links (NVLink alias)", "counter",
         [(lbl(g), xsum(g, 0)) for g in gpus])
    emit("DCGM_FI_PROF_NVLINK_TX_BYTES", "xGMI bytes written, all links (NVLink alias)",
         "counter", [(lbl(g), xsum(g, 1)) for g in gpus])
    emit("amd_gpu_exporter_gpus", "GPUs found", "gauge", [({"Hostname": node}, len(gpus))])
    return "\n".join(L) + "\n"


class Exporter:
    def __init__(self, sysfs_root: str = "/sys", node: Optional[str] = None, ttl: float = 1.0,
                 run=_run_amdsmi, smi_ttl: float = 5.0):
        self.root = sysfs_root
        self.node = node or os.environ.get("NODE_NAME") or socket.gethostname()
        self.ttl = ttl
        self.run = run
        self.smi_ttl = smi_ttl  # amd-smi calls take ~1 s: refreshed less often than sysfs
        self._smi = (0.0, [], {})
        self._cache = (0.0, "")
        self._lock = threading.Lock()

    def _amdsmi(self):
        t, metric, xgmi = self._smi
        if time.time() - t > self.smi_ttl:
            metric, xgmi = read_amdsmi(self.run), read_xgmi(self.run)
            self._smi = (time.time(), metric, xgmi)
        return metric, xgmi

    def collect(self) -> list[dict]:
        gpus = read_sysfs(self.root)
        metric, xgmi = self._amdsmi()
        if not gpus:
            gpus = metric
            for g in gpus:
                if g["gpu"] in xgmi:
                    g["xgmi"] = xgmi[g["gpu"]]
            return gpus
        # sysfs first; amd-smi fills what the sysfs tree lacks, matched by PCI bus id (amd-smi
        # numbers only the GPUs this process can see); by index only when no bus ids exist
        by_pci = {g["pci"].lower(): g for g in gpus if _BUS.match(str(g.get("pci", "")).lower())}

        def find(idx, pci):
            if by_pci and pci:
                return by_pci.get(pci)
            return next((x for x in gpus if x["gpu"] == idx), None)

        for m in metric:  # no `amd-smi list` mapping: the xgmi report names bus ids too
            g = find(m["gpu"], m.get("pci") or xgmi.get(m["gpu"], {}).get("pci", ""))
            if g is None:
                continue
            for k in ("clocks", "ecc"):
                if not g.get(k) and m.get(k):
                    g[k] = m[k]
            for k in ("pcie_replay", "energy_j", "xgmi_err"):
                if g.get(k) is None and m.get(k) is not None:
                    g[k] = m[k]
        for idx, x in xgmi.items():
            g = find(idx, x.get("pci", ""))
            if g is not None:
                g["xgmi"] = x
        return gpus

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
