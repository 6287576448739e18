"""Per-rank telemetry of multi-process engine pods on ONE /metrics endpoint.

A TP engine is N processes (torchrun) but only rank 0 serves HTTP.  Every follower rank runs
its own in-process telemetry (kernel-stats windows, GPU counters: exporter/inprocess_profiler,
exporter/pmc_sampler) with a `rank` label and writes the rendered text to a file under
/dev/shm (shared by the processes of the pod) every few seconds; rank 0 merges the files of its
group into its /metrics.  The merge keeps Prometheus text-format rules: one HELP / TYPE per
metric family, all of a family's samples together.
"""
from __future__ import annotations

import os
import re
import threading
import time
from typing import Callable, Optional

DIR = os.environ.get("AKAP_RANK_METRICS_DIR", "/dev/shm/akap-metrics")
STALE_S = 300.0

_SAMPLE = re.compile(r"^([a-zA-Z_:][a-zA-Z0-9_:]*)(\{[^}]*\})?(\s+.*)$")


def add_labels(text: str, labels: dict) -> str:
    """Add labels to every sample line of a Prometheus text block."""
    if not labels:
        return text
    extra = ",".join(f'{k}="{v}"' for k, v in sorted(labels.items()))
    out = []
    for line in text.splitlines():
        m = _SAMPLE.match(line) if line and not line.startswith("#") else None
        if m is None:
            out.append(line)
            continue
        name, lab, rest = m.group(1), m.group(2), m.group(3)
        lab = "{" + extra + "}" if not lab or lab == "{}" else lab[:-1] + "," + extra + "}"
        out.append(name + lab + rest)
    return "\n".join(out) + ("\n" if text.endswith("\n") else "")


def _family(name: str, declared: set) -> str:
    for suf in ("_bucket", "_count", "_sum", "_total", "_created"):
        if name.endswith(suf) and name[: -len(suf)] in declared:
            return name[: -len(suf)]
    return name


def merge(texts: list) -> str:
    """Merge Prometheus text blocks: one HELP / TYPE per family, its samples together."""
    order: list = []
    meta: dict = {}
    samples: dict = {}
    for text in texts:
        declared: set = set()
        for line in text.splitlines():
            if not line.strip():
                continue
            if line.startswith("#"):
                parts = line.split(None, 3)
                if len(parts) >= 3 and parts[1] in ("HELP", "TYPE"):
                    fam = parts[2]
                    declared.add(fam)
                    if fam not in meta:
                        meta[fam] = {}
                        order.append(fam)
                    meta[fam].setdefault(parts[1], line)
                continue
            m = _SAMPLE.match(line)
            if m is None:
                continue
            fam = _family(m.group(1), declared)
            if fam not in meta:
                meta[fam] = {}
                order.append(fam)
            samples.setdefault(fam, []).append(line)
    out = []
    for fam in order:
        for k in ("HELP", "TYPE"):
            if k in meta[fam]:
                out.append(meta[fam][k])
        out += samples.get(fam, [])
    return "\n".join(out) + "\n" if out else ""


def _path(tag: str, rank: int) -> str:
    safe = re.sub(r"[^A-Za-z0-9_.-]", "_", tag)
    return os.path.join(DIR, f"{safe}-rank{rank}.prom")


class RankMetricsWriter:
    """Follower rank: render `providers` every `interval_s` into this rank's file."""

    def __init__(self, tag: str, rank: int, providers: list, interval_s: float = 5.0):
        self.tag, self.rank = tag, rank
        self.providers: list[Callable[[], str]] = providers
        self.interval_s = interval_s
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.writes = 0

    def write_once(self) -> None:
        text = merge([p() for p in self.providers])
        os.makedirs(DIR, exist_ok=True)
        path = _path(self.tag, self.rank)
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            f.write(text)
        os.replace(tmp, path)
        self.writes += 1

    def _loop(self) -> None:
        while not self._stop.wait(self.interval_s):
            try:
                self.write_once()
            except OSError:
                pass

    def start(self) -> "RankMetricsWriter":
        self._thread = threading.Thread(target=self._loop, name="rank-metrics", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()


def read_peers(tag: str, exclude_rank: int = 0) -> list:
    """Texts the other ranks of group `tag` wrote (stale files ignored)."""
    if not os.path.isdir(DIR):
        return []
    prefix = re.sub(r"[^A-Za-z0-9_.-]", "_", tag) + "-rank"
    out, now = [], time.time()
    for name in sorted(os.listdir(DIR)):
        if not (name.startswith(prefix) and name.endswith(".prom")):
            continue
        if name == os.path.basename(_path(tag, exclude_rank)):
            continue
        path = os.path.join(DIR, name)
        try:
            if now - os.path.getmtime(path) > STALE_S:
                continue
            with open(path) as f:
                out.append(f.read())
        except OSError:
            continue
    return out
