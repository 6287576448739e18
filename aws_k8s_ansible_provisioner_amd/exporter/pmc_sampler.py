"""GPU hardware counters (rocprofiler-sdk device counting service) on the engine's /metrics.

The counters come from `libakap_pmc.so` (csrc/tools/pmc_tool.cpp), a rocprofiler-sdk tool
that the ROCm runtime loads at process start when ROCP_TOOL_LIBRARIES names it (the engine
pods set it; `python -m aws_k8s_ansible_provisioner_amd.server --pmc-interval 5`).  The tool
configures the device counting service on each GPU agent; this module reads the counters every
`interval` seconds through the tool's C ABI and serves, per counter, its rate since the
previous read, plus derived series:

  akap_gpu_pmc_up                              1 while reads succeed
  akap_gpu_pmc_rate{counter="SQ_WAVES"}        events per second, every collected counter
  akap_gpu_pmc_gpu_busy_ratio                  GRBM_GUI_ACTIVE / GRBM_COUNT
  akap_gpu_pmc_mfma_busy_ratio                 SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x CUs per
                                               XCD x 4 SIMDs): GRBM counters are summed over the
                                               8 XCDs, MFMA busy over every SIMD.  Calibrated on
                                               back-to-back 8192^3 bf16 matmuls at 1.37 PFLOP/s:
                                               0.68, vs 0.64 of the clock-scaled peak
                                               (profiles/r4_pmc_probe.log)
  akap_gpu_pmc_mem_read_bytes_per_second       TCC_EA0_RDREQ x 128 B (memory-side reads: HBM +
                                               Infinity Cache; 128-B requests, the calibration of
                                               profiles/r3_pmc_calibrated_decode.md)
  akap_gpu_pmc_mem_write_bytes_per_second      TCC_EA0_WRREQ x 64 B
  akap_gpu_pmc_lds_bank_conflict_rate          SQ_LDS_BANK_CONFLICT cycles per second

No ptrace, no sidecar, no dispatch serialisation: unlike `rocprofv3 --pmc` (dispatch counting),
device counting reads agent-wide counters between two points in time, so it stays on under
serving load and sees hipGraph replays.  The reference's equivalent contract is the DCGM
exporter scrape + its PromQL probes (otel-observability-setup.yaml:393-468,735-743).
"""
from __future__ import annotations

import ctypes
import os
import threading
import time
from typing import Optional

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(PKG, "libakap_pmc.so")
SIMDS_PER_CU = 4
CUS_PER_XCD = int(os.environ.get("AKAP_PMC_CUS_PER_XCD", "32"))  # MI355X: 256 CUs / 8 XCDs


def tool_env() -> dict:
    """Environment that makes the ROCm runtime load the counter tool at process start."""
    return {"ROCP_TOOL_LIBRARIES": LIB}


class PMCSampler:
    def __init__(self, interval_s: float = 5.0, agent: int = 0, lib: Optional[str] = None,
                 labels: Optional[dict] = None):
        self.interval_s = interval_s
        self.agent = agent
        self.labels = dict(labels or {})
        self.path = lib or os.environ.get("ROCP_TOOL_LIBRARIES", LIB).split(":")[0]
        self._lib = None
        self.names: list[str] = []
        self.rates: dict[str, float] = {}
        self.reads = 0
        self.failures = 0
        self.last_error: Optional[str] = None
        self._prev: Optional[list] = None
        self._t_prev = 0.0
        self.cumulative: Optional[bool] = None
        self.settle_s = 0.1
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    # ------------------------------------------------------------------ tool access
    def _open(self):
        if self._lib is None:
            lib = ctypes.CDLL(self.path)  # the instance the runtime loaded (same path)
            lib.akap_pmc_status.restype = ctypes.c_char_p
            lib.akap_pmc_name.restype = ctypes.c_char_p
            lib.akap_pmc_sample.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                            ctypes.c_int]
            self._lib = lib
        return self._lib

    def status(self) -> str:
        try:
            return self._open().akap_pmc_status().decode()
        except OSError as e:
            return f"tool library not loadable: {e}"

    def _read(self) -> list:
        lib = self._open()
        n = lib.akap_pmc_count(self.agent)
        if n <= 0:
            raise RuntimeError(f"no counters ({lib.akap_pmc_status().decode()})")
        if not self.names:
            self.names = [lib.akap_pmc_name(self.agent, i).decode() for i in range(n)]
        buf = (ctypes.c_double * n)()
        got = lib.akap_pmc_sample(self.agent, buf, n)
        if got < 0:
            raise RuntimeError(lib.akap_pmc_status().decode())
        return list(buf[:got])

    def once(self) -> bool:
        try:
            vals = self._read()
            now = time.monotonic()
            if self.cumulative is None:
                # the first read starts the counting context (values ~0): let the counters run
                # for a moment, then two back-to-back reads tell the service's semantics apart
                # -- cumulative counters barely move in between, per-read (reset) counters
                # restart near 0
                time.sleep(self.settle_s)
                vals = self._read()
                again = self._read()
                now = time.monotonic()
                big = [i for i, v in enumerate(vals) if v > 1e6]
                self.cumulative = bool(big) and all(again[i] >= 0.5 * vals[i] for i in big)
                vals = again
            with self._lock:
                if self._prev is not None and now > self._t_prev:
                    dt = now - self._t_prev
                    deltas = [(v - p if self.cumulative else v) for v, p in zip(vals, self._prev)]
                    self.rates = {n: max(d, 0.0) / dt for n, d in zip(self.names, deltas)}
                self._prev, self._t_prev = vals, now
                self.reads += 1
                self.last_error = None
            return True
        except Exception as e:  # a counter failure must never take the engine down
            with self._lock:
                self.failures += 1
                self.last_error = f"{type(e).__name__}: {e}"[:300]
            return False

    def _loop(self) -> None:
        self.once()
        while not self._stop.wait(self.interval_s):
            self.once()

    def start(self) -> "PMCSampler":
        self._thread = threading.Thread(target=self._loop, name="pmc-sampler", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()

    # ------------------------------------------------------------------ exposition
    def derived(self) -> dict:
        r = self.rates
        out = {}
        if r.get("GRBM_COUNT"):
            out["gpu_busy_ratio"] = r.get("GRBM_GUI_ACTIVE", 0.0) / r["GRBM_COUNT"]
        if r.get("GRBM_GUI_ACTIVE"):
            out["mfma_busy_ratio"] = min(1.0, r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) /
                                         (r["GRBM_GUI_ACTIVE"] * CUS_PER_XCD * SIMDS_PER_CU))
        if "TCC_EA0_RDREQ_sum" in r:
            out["mem_read_bytes_per_second"] = r["TCC_EA0_RDREQ_sum"] * 128.0
        if "TCC_EA0_WRREQ_sum" in r:
            out["mem_write_bytes_per_second"] = r["TCC_EA0_WRREQ_sum"] * 64.0
        if "SQ_LDS_BANK_CONFLICT" in r:
            out["lds_bank_conflict_rate"] = r["SQ_LDS_BANK_CONFLICT"]
        return out

    def text(self) -> str:
        with self._lock:
            rates, ok, bad, err = dict(self.rates), self.reads, self.failures, self.last_error
            derived = self.derived()
        def lab(**extra) -> str:  # the label set of one sample ("" when empty)
            items = sorted(self.labels.items()) + sorted(extra.items())
            return "{" + ",".join(f'{k}="{v}"' for k, v in items) + "}" if items else ""

        lines = ["# HELP akap_gpu_pmc_up 1 if the newest GPU counter read succeeded",
                 "# TYPE akap_gpu_pmc_up gauge",
                 f"akap_gpu_pmc_up{lab()} {1 if ok and err is None else 0}",
                 "# HELP akap_gpu_pmc_reads_total GPU counter reads by result",
                 "# TYPE akap_gpu_pmc_reads_total counter",
                 f"akap_gpu_pmc_reads_total{lab(result='ok')} {ok}",
                 f"akap_gpu_pmc_reads_total{lab(result='failed')} {bad}"]
        if rates:
            lines += ["# HELP akap_gpu_pmc_rate GPU hardware counter events per second "
                      "(rocprofiler-sdk device counting)", "# TYPE akap_gpu_pmc_rate gauge"]
            lines += [f"akap_gpu_pmc_rate{lab(counter=n)} {v:.6g}" for n, v in sorted(rates.items())]
        for k, v in sorted(derived.items()):
            lines += [f"# TYPE akap_gpu_pmc_{k} gauge", f"akap_gpu_pmc_{k}{lab()} {v:.6g}"]
        return "\n".join(lines) + "\n"
