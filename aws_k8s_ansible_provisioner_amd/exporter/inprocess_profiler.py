"""In-process kernel-stats windows: the engine samples its OWN GPU kernels with torch.profiler
(roctracer / rocprofiler underneath on ROCm) and serves them on its /metrics as the same
akap_kernel_* series the rocprofv3 --attach sidecar (kernel_profiler.py) produces.

Why a second path: the sidecar needs ptrace on the engine (shareProcessNamespace +
CAP_SYS_PTRACE), which a locked-down node may refuse -- the MI355X box this repo is measured
on answers EPERM (profiles/r3_observability_gpu_box.md).  An in-process window needs no
privileges and sees every kernel, hipGraph replays included (profiles/r3_inprocess_kprof.log).
Cost: roctracer is on only during a window (default 1 s every 60 s); closing a window parses
its events on the profiler thread (~1-2 s of host time that shares the GIL with the engine
loop), so the interval should stay long.

    python -m aws_k8s_ansible_provisioner_amd.server ... --kernel-stats-interval 60
"""
from __future__ import annotations

import threading
import time
from typing import Callable, Optional

from . import rocprof_bridge

WindowFn = Callable[[float], dict]


def torch_window(window_s: float) -> dict:
    """One profiling window of this process: {kernel name: (device seconds, calls)}."""
    import torch
    from torch.profiler import ProfilerActivity, profile

    if not torch.cuda.is_available():  # no GPU: no kernels to see (a CPU engine)
        time.sleep(window_s)
        return {}

    p = profile(activities=[ProfilerActivity.CUDA])
    p.start()
    time.sleep(window_s)
    p.stop()
    out: dict = {}
    for e in p.events():
        if getattr(e.device_type, "name", "") != "CUDA":
            continue
        us = getattr(e, "device_time_total", None)
        if us is None:
            us = e.cuda_time_total
        t, n = out.get(e.name, (0.0, 0))
        out[e.name] = (t + us * 1e-6, n + 1)
    return out


class InProcessKernelProfiler:
    def __init__(self, window_ms: int = 1000, interval_s: float = 60.0, keep: int = 8,
                 window_fn: Optional[WindowFn] = None):
        self.window_s = window_ms / 1000.0
        self.interval_s = interval_s
        self.keep = keep
        self.window_fn = window_fn or torch_window
        self.windows: list[dict] = []
        self.ok = 0
        self.failures = 0
        self.last_error: Optional[str] = None
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def once(self) -> bool:
        try:
            w = self.window_fn(self.window_s)
        except Exception as e:  # a profiler failure must never take the engine down
            with self._lock:
                self.failures += 1
                self.last_error = f"{type(e).__name__}: {e}"[:300]
            return False
        with self._lock:
            self.windows = (self.windows + [w])[-self.keep:]
            self.ok += 1
            self.last_error = None
        return True

    def _loop(self) -> None:
        while not self._stop.wait(self.interval_s):
            self.once()

    def start(self) -> "InProcessKernelProfiler":
        self._thread = threading.Thread(target=self._loop, name="kernel-stats", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()

    def text(self) -> str:
        with self._lock:
            wins, ok, bad = list(self.windows), self.ok, self.failures
            up = 1 if (ok and self.last_error is None) else 0
        body = rocprof_bridge.render_aggregates(wins, self.window_s) if wins else ""
        return body + "\n".join([
            "# HELP akap_kernel_profiler_up 1 if the newest profiling window succeeded",
            "# TYPE akap_kernel_profiler_up gauge", f"akap_kernel_profiler_up {up}",
            "# HELP akap_kernel_profiler_windows_total Profiling windows by result",
            "# TYPE akap_kernel_profiler_windows_total counter",
            f'akap_kernel_profiler_windows_total{{result="ok"}} {ok}',
            f'akap_kernel_profiler_windows_total{{result="failed"}} {bad}']) + "\n"
