"""Endpoint picker (the llm-d "EPP"): chooses the model-server pod for each request.

Scoring (higher is better), per candidate endpoint e:
  queue    = 1 / (1 + waiting_e + 0.25 * running_e + inflight_e)      (load)
  kv       = 1 - kv_usage_e                                            (KV headroom)
  prefix   = matched_prefix_blocks_e / request_blocks                   (cache affinity)
  score    = w_queue * queue + w_kv * kv + w_prefix * prefix
Endpoints that are unhealthy, or whose metrics are stale, are filtered out.  The prefix
index is the gateway's own memory of which endpoint served which prompt-prefix block
hashes (same chained-hash scheme as the engine's prefix cache, computed on the prompt
text in fixed-size character blocks), so routing is cache-aware without asking pods.

Disaggregated prefill/decode: with both roles present and a prompt of at least
`pd_threshold` characters, `pick_pd` returns a (prefill, decode) pair; pairs whose decode
endpoint pulls KV by hipIpc (akap:kv_transport_ipc) get `w_ipc` on top of their score.  A prefill and a decode
endpoint can only be paired inside one P/D transfer group (the torch.distributed / RCCL group
their processes share -- in the `pd` preset, the two processes of one pod), so every endpoint
carries a `group` and the pair is the best-scoring (prefill + decode) within a group.
"""
from __future__ import annotations

import dataclasses
import hashlib
import random
import threading
import time
from collections import OrderedDict
from typing import Optional


@dataclasses.dataclass
class Endpoint:
    url: str
    role: str = "both"  # both | prefill | decode
    group: str = ""     # P/D transfer group (prefill and decode pair only within one)
    healthy: bool = True
    running: float = 0.0
    waiting: float = 0.0
    kv_usage: float = 0.0
    inflight: int = 0
    last_scrape: float = 0.0
    failures: int = 0
    served: int = 0
    kv_broken: bool = False  # P/D: its KV-transfer channel awaits a rebuild
    kv_ipc: bool = False     # P/D decode: pulls KV by hipIpc (no peer fell back to p2p)

    def load_score(self) -> float:
        return 1.0 / (1.0 + self.waiting + 0.25 * self.running + self.inflight)


def prefix_hashes(text: str, block_chars: int = 64, max_blocks: int = 64) -> list[int]:
    hs, parent = [], b""
    n = min(len(text) // block_chars, max_blocks)
    for i in range(n):
        h = hashlib.blake2b(parent + text[i * block_chars:(i + 1) * block_chars].encode(),
                            digest_size=8).digest()
        hs.append(int.from_bytes(h, "little"))
        parent = h
    return hs


class PrefixIndex:
    """LRU map: prefix-block hash -> endpoint url."""

    def __init__(self, capacity: int = 200_000):
        self.cap = capacity
        self.map: OrderedDict[int, str] = OrderedDict()
        self.lock = threading.Lock()

    def match(self, hashes: list[int]) -> dict[str, int]:
        """Per endpoint: number of leading prefix blocks it is known to hold."""
        out: dict[str, int] = {}
        with self.lock:
            for i, h in enumerate(hashes):
                url = self.map.get(h)
                if url is None:
                    break
                self.map.move_to_end(h)
                out[url] = i + 1
        return out

    def insert(self, hashes: list[int], url: str) -> None:
        with self.lock:
            for h in hashes:
                self.map[h] = url
                self.map.move_to_end(h)
            while len(self.map) > self.cap:
                self.map.popitem(last=False)


@dataclasses.dataclass
class PickerConfig:
    w_queue: float = 1.0
    w_kv: float = 1.0
    w_prefix: float = 2.0
    w_ipc: float = 1.0  # P/D pairs whose decode side pulls KV by hipIpc (xGMI / same GPU)
    stale_after_s: float = 15.0
    pd_threshold_chars: int = 512
    block_chars: int = 64


class EndpointPicker:
    def __init__(self, endpoints: list[Endpoint], cfg: Optional[PickerConfig] = None,
                 seed: int = 0):
        self.cfg = cfg or PickerConfig()
        self.eps: dict[str, Endpoint] = {e.url: e for e in endpoints}
        self.prefix = PrefixIndex()
        self.rng = random.Random(seed)
        self.lock = threading.Lock()

    # ---------------------------------------------------------------- membership
    def set_endpoints(self, urls_roles: list[tuple]) -> None:
        """(url, role) or (url, role, group); the default group is the URL's host (the two
        P/D processes of one pod share its IP)."""
        with self.lock:
            keep = {}
            for item in urls_roles:
                url, role = item[0], item[1]
                group = item[2] if len(item) > 2 and item[2] else default_group(url)
                keep[url] = self.eps.get(url) or Endpoint(url, role, group)
                keep[url].role = role
                keep[url].group = group
            self.eps = keep

    def endpoints(self) -> list[Endpoint]:
        return list(self.eps.values())

    def update_metrics(self, url: str, running: float, waiting: float, kv: float,
                       kv_broken: bool = False, kv_ipc: bool = False) -> None:
        e = self.eps.get(url)
        if e is None:
            return
        e.running, e.waiting, e.kv_usage = running, waiting, kv
        e.kv_broken = kv_broken
        e.kv_ipc = kv_ipc
        e.last_scrape = time.time()
        e.healthy = True
        e.failures = 0

    def mark_failure(self, url: str, hard: bool = False) -> None:
        e = self.eps.get(url)
        if e is None:
            return
        e.failures += 1
        if hard or e.failures >= 3:
            e.healthy = False

    # ---------------------------------------------------------------- scoring
    def _candidates(self, roles: tuple[str, ...]) -> list[Endpoint]:
        now = time.time()
        c = [e for e in self.eps.values() if e.healthy and e.role in roles and
             (e.last_scrape == 0.0 or now - e.last_scrape < self.cfg.stale_after_s)]
        if not c:  # degrade gracefully: anything healthy in the role set
            c = [e for e in self.eps.values() if e.healthy and e.role in roles]
        return c

    def score(self, e: Endpoint, prefix_match: dict[str, int], nblocks: int) -> float:
        cfg = self.cfg
        p = (prefix_match.get(e.url, 0) / nblocks) if nblocks else 0.0
        return (cfg.w_queue * e.load_score() + cfg.w_kv * (1.0 - e.kv_usage)
                + cfg.w_prefix * p)

    def pick(self, prompt_text: str = "", roles: tuple[str, ...] = ("both",)) -> Optional[Endpoint]:
        cands = self._candidates(roles)
        if not cands:
            return None
        hs = prefix_hashes(prompt_text, self.cfg.block_chars)
        match = self.prefix.match(hs)
        best, best_s = [], -1e30
        for e in cands:
            s = self.score(e, match, len(hs))
            if s > best_s + 1e-9:
                best, best_s = [e], s
            elif abs(s - best_s) <= 1e-9:
                best.append(e)
        chosen = self.rng.choice(best)
        if hs:
            self.prefix.insert(hs, chosen.url)
        chosen.served += 1
        return chosen

    def pick_pd(self, prompt_text: str, pd_ok: bool = True
                ) -> tuple[Optional[Endpoint], Optional[Endpoint]]:
        """(prefill, decode) for disaggregated serving, or (None, endpoint) when the
        request should run monolithically (short prompt, n > 1 / several prompts, or no
        transfer group with a healthy prefill AND decode endpoint)."""
        if pd_ok and len(prompt_text) >= self.cfg.pd_threshold_chars:
            pre = self._candidates(("prefill",))
            dec = self._candidates(("decode",))
            if pre and dec:
                hs = prefix_hashes(prompt_text, self.cfg.block_chars)
                match = self.prefix.match(hs)
                best, best_s = None, -1e30
                for p in pre:
                    for d in dec:
                        if p.group != d.group or p.kv_broken or d.kv_broken:
                            continue  # other transfer group, or a channel being rebuilt
                        s = self.score(p, match, len(hs)) + self.score(d, {}, 0)
                        if d.kv_ipc:  # the hipIpc pull beats any send/recv path
                            s += self.cfg.w_ipc
                        if s > best_s + 1e-9 or (abs(s - best_s) <= 1e-9 and
                                                 self.rng.random() < 0.5):
                            best, best_s = (p, d), s
                if best is not None:
                    if hs:
                        self.prefix.insert(hs, best[0].url)
                    best[0].served += 1
                    best[1].served += 1
                    return best
        return None, self.pick(prompt_text, ("both", "decode"))


def default_group(url: str) -> str:
    from urllib.parse import urlparse

    return urlparse(url).hostname or url


def parse_prometheus(text: str) -> dict[str, float]:
    """Sum samples per metric name (labels dropped) from Prometheus text format."""
    out: dict[str, float] = {}
    for line in text.splitlines():
        if not line or line[0] == "#":
            continue
        try:
            name_part, val = line.rsplit(" ", 1)
            name = name_part.split("{", 1)[0]
            out[name] = out.get(name, 0.0) + float(val)
        except ValueError:
            continue
    return out
