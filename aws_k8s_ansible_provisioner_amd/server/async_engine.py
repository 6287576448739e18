"""Asyncio front of the engine: one background thread drives LLMEngine.step() while
HTTP handlers await per-request output queues.

The step loop never blocks the event loop (GPU work + the C++ scheduler run in the
engine thread; outputs are handed over with call_soon_threadsafe).  When idle the
thread parks on an Event, so an idle pod burns no CPU.
"""
from __future__ import annotations

import asyncio
import dataclasses
import json
import os
import queue
import threading
import urllib.request
import time
import traceback
from typing import AsyncIterator, Optional

from ..engine.config import SamplingParams
from ..engine.llm_engine import LLMEngine, RequestOutput
from ..parallel.kv_transfer import KVIpcOpenTimeout


class EngineDeadError(RuntimeError):
    pass


class KVTransferError(RuntimeError):
    """P/D: the prefill pod could not hand the request's KV over (pod gone, timeout,
    block-count mismatch).  The decode side frees its reserved blocks and fails the
    request; the gateway may retry it monolithically."""


@dataclasses.dataclass
class PullJob:
    req_id: str
    prompt_ids: list
    first: int
    params: SamplingParams
    stream: bool
    kvp: dict
    fut: "asyncio.Future"
    loop: "asyncio.AbstractEventLoop"


def decode_transport(kv_agent) -> str:
    """AKAP_KV_TRANSPORT: ipc (GPU default: pull the blocks out of the prefill engine's
    hipIpc-mapped cache) or p2p (/kv/push + a packed send/recv over the process group)."""
    env = os.environ.get("AKAP_KV_TRANSPORT", "auto")
    if env in ("ipc", "p2p"):
        return env
    return "ipc" if getattr(kv_agent, "is_gpu", False) else "p2p"


class KVPuller:
    """Decode-side P/D data path.  Pulls queued at the same moment from the same prefill
    server are coalesced: blocks are reserved for each request, ONE POST /kv/push names all
    their transfer ids, and ONE packed RCCL recv lands every request's KV (the prefill side
    gathers all their blocks into one send), instead of one HTTP round trip + one P2P
    transfer per request."""

    MAX_BATCH = 64

    def __init__(self, ae: "AsyncEngine"):
        self.ae = ae
        self.q: "queue.Queue[PullJob]" = queue.Queue()
        self.batches = 0
        self.ipc_fallback: set = set()  # prefill URLs whose cache could not be mapped
        self._thread = threading.Thread(target=self._run, name="kv-puller", daemon=True)
        self._thread.start()

    def submit(self, job: PullJob) -> None:
        self.q.put(job)

    @staticmethod
    def _resolve(job: PullJob, err: Optional[BaseException]) -> None:
        def set_():
            if job.fut.done():
                return
            if err is None:
                job.fut.set_result(True)
            else:
                job.fut.set_exception(err)

        job.loop.call_soon_threadsafe(set_)

    def _run(self) -> None:
        while True:
            jobs = [self.q.get()]
            time.sleep(0.001)  # let concurrent pulls of the same moment join the batch
            while len(jobs) < self.MAX_BATCH:
                try:
                    jobs.append(self.q.get_nowait())
                except queue.Empty:
                    break
            groups: dict = {}
            for j in jobs:
                groups.setdefault((j.kvp["remote_url"], int(j.kvp["remote_rank"])),
                                  []).append(j)
            for (url, rank), js in groups.items():
                self._pull_batch(url, rank, js)

    def _pull_batch(self, url: str, rank: int, jobs: list) -> None:
        eng = self.ae.engine
        ready, reserved = [], []
        for j in jobs:
            try:
                iid, blocks = eng.reserve_prefilled(j.req_id, j.prompt_ids, j.first, j.params,
                                                    j.stream)
                if not blocks:
                    raise RuntimeError("KV pool exhausted on the decode engine")
                ready.append(j)
                reserved.append((iid, blocks))
            except Exception as e:
                AsyncEngine._release_remote(j.kvp)
                self._resolve(j, e)
        if not ready:
            return
        leased = None
        if self.transport() == "ipc" and url not in self.ipc_fallback:
            leased = self._pull_batch_ipc(url, ready, reserved)
            if leased is True:
                return
            # the peer cache could not be mapped in time: this and every later batch from
            # this prefill server move over the process group instead (the leased blocks of
            # this batch are pushed as they are)
            self.ipc_fallback.add(url)
        self._pull_batch_p2p(url, rank, ready, reserved, leased)

    def _pull_batch_p2p(self, url: str, rank: int, ready: list, reserved: list,
                        leased: Optional[list] = None) -> None:
        eng = self.ae.engine
        agent = self.ae.kv_agent
        try:
            msg = {"transfer_ids": [int(j.kvp["transfer_id"]) for j in ready],
                   "dst_rank": eng.rank, "group": self.ae.pd_group}
            if self.ae.pd_bootstrap == "http":
                # two-pod P/D: this prefill server's own pair channel (we are its rank 1)
                agent = self.ae.pair_agent(url)
                msg["peer"] = self.ae.peer_id()
                msg["dst_rank"], rank = 1, 0
            if leased is not None:
                msg["leased_blocks"] = leased
            body = json.dumps(msg).encode()
            req = urllib.request.Request(url.rstrip("/") + "/kv/push", data=body,
                                         headers={"Content-Type": "application/json"})
            with urllib.request.urlopen(req, timeout=60) as r:
                meta = json.loads(r.read())
            counts = [int(n) for n in meta.get("num_blocks", [])]
            if counts != [len(b) for _, b in reserved]:
                raise RuntimeError(f"KV block count mismatch {counts} vs "
                                   f"{[len(b) for _, b in reserved]}")
            all_blocks = [b for _, bl in reserved for b in bl]
            agent.recv_blocks(all_blocks, rank)
        except Exception as e:
            for j, (iid, _) in zip(ready, reserved):
                eng.abort_request(j.req_id)  # frees the reserved decode blocks
                AsyncEngine._release_remote(j.kvp)
                self._resolve(j, e)
            if self.ae.pd_bootstrap == "http":
                # a pair channel is not reset in place: the next batch forms a new one
                with self.ae._pair_lock:
                    ag = self.ae.pair_agents.pop(url, None)
                if ag is not None:
                    ag.close()
                return
            if (getattr(agent, "broken", None) is not None or
                    "KVChannelBroken" in _http_error_text(e)):
                # a timed-out transfer left stale ops in the channel (ours or the prefill
                # side's): rebuild it on both sides so the NEXT request on this pair works
                self.ae.rebuild_channel(url)
            return
        self.batches += 1
        for j, (iid, _) in zip(ready, reserved):
            eng.activate(iid)
            self._resolve(j, None)
        self.ae._wake.set()


    def transport(self) -> str:
        return decode_transport(self.ae.kv_agent)

    def _pull_batch_ipc(self, url: str, ready: list, reserved: list):
        """hipIpc transport: lease the transfers' blocks (POST /kv/lease), map the prefill
        cache on first use, ONE kv_pull launch moves every request's blocks and fills their V
        tails, then release the lease (POST /kv/done) -- also on failure.  Returns True when
        the batch is resolved; when the peer cache could not be mapped within
        AKAP_IPC_OPEN_TIMEOUT_S it returns the leased prefill block lists (nothing resolved,
        the decode blocks still reserved): the caller pushes them over the p2p transport."""
        eng = self.ae.engine
        agent = self.ae.kv_agent
        runner = eng.runner
        tids = [int(j.kvp["transfer_id"]) for j in ready]

        def post(path, body):
            req = urllib.request.Request(url.rstrip("/") + path, data=json.dumps(body).encode(),
                                         headers={"Content-Type": "application/json"})
            with urllib.request.urlopen(req, timeout=60) as r:
                return json.loads(r.read())

        leased = False
        try:
            meta = post("/kv/lease", {"transfer_ids": tids})
            leased = True
            src = [[int(b) for b in bl] for bl in meta["blocks"]]
            if [len(b) for b in src] != [len(b) for _, b in reserved]:
                raise RuntimeError(f"KV block count mismatch {[len(b) for b in src]} vs "
                                   f"{[len(b) for _, b in reserved]}")
            peer = agent.connect_ipc(meta["ipc"])  # one mapping per prefill engine
            bs = eng.ecfg.block_size
            pairs, tails = [], []
            for j, (iid, blocks), sb in zip(ready, reserved, src):
                pairs += list(zip(sb, blocks))
                n = len(j.prompt_ids)
                if runner.v_tails is not None and n % 8:
                    slot = eng.tail_slot(iid)
                    if slot >= 0:
                        g0 = n & ~7
                        tails.append((sb[g0 // bs], (g0 % bs) // 8, n % 8, slot))
            agent.pull(pairs, runner.model.hkv, bs, runner.model.D,
                       tail=getattr(runner, "_tail", None), tail_jobs=tails, peer=peer)
        except KVIpcOpenTimeout as e:
            print(f"[pd] {e}: KV from {url} moves over the p2p transport", flush=True)
            return src
        except Exception as e:
            for j, (iid, _) in zip(ready, reserved):
                eng.abort_request(j.req_id)  # frees the reserved decode blocks
                if not leased:
                    AsyncEngine._release_remote(j.kvp)
                self._resolve(j, e)
            if leased:
                try:
                    post("/kv/done", {"transfer_ids": tids})
                except Exception as e2:  # the prefill side's TTL cannot free leased blocks
                    print(f"[pd] /kv/done to {url} failed: {e2}", flush=True)
            return True
        try:
            post("/kv/done", {"transfer_ids": tids})
        except Exception as e:
            print(f"[pd] /kv/done to {url} failed: {e}", flush=True)
        self.batches += 1
        for j, (iid, _) in zip(ready, reserved):
            eng.activate(iid, tail_filled=True)
            self._resolve(j, None)
        self.ae._wake.set()
        return True


def _http_error_text(e: BaseException) -> str:
    """Body of an urllib HTTPError (the server's JSON error), else the exception text."""
    try:
        return e.read().decode()  # type: ignore[attr-defined]
    except Exception:
        return str(e)


class AsyncEngine:
    def __init__(self, engine: LLMEngine, step_hook=None):
        self.engine = engine
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.queues: dict[str, asyncio.Queue] = {}
        self._wake = threading.Event()
        self._stop = False
        self.dead: Optional[str] = None
        self.step_hook = step_hook
        self.kv_agent = None  # parallel.kv_transfer.KVTransferAgent for P/D roles
        self.pd_group: Optional[str] = None  # P/D: id of this engine's RCCL transfer group
        self.pd_bootstrap = "launcher"  # "http": two-pod P/D, pair channels on demand
        self.pair_host = None           # prefill (http): kv_transfer.PairHost
        self.pair_agents: dict = {}     # decode (http): prefill URL -> pair KVTransferAgent
        self._pair_gen = 0
        self._pair_lock = threading.Lock()
        self.puller: Optional["KVPuller"] = None
        self._thread = threading.Thread(target=self._run, name="engine-loop", daemon=True)
        self.started = time.time()

    def start(self, loop: Optional[asyncio.AbstractEventLoop] = None) -> None:
        self.loop = loop or asyncio.get_event_loop()
        self._thread.start()

    def stop(self) -> None:
        self._stop = True
        self._wake.set()

    @property
    def healthy(self) -> bool:
        return self.dead is None and self._thread.is_alive()

    def _deliver(self, outs: list[RequestOutput]) -> None:
        for o in outs:
            q = self.queues.get(o.req_id)
            if q is not None:
                self.loop.call_soon_threadsafe(q.put_nowait, o)

    def _run(self) -> None:
        eng = self.engine
        try:
            while not self._stop:
                if not eng.has_unfinished():
                    self._wake.wait(0.05)
                    self._wake.clear()
                    continue
                outs = eng.step()
                if self.step_hook is not None:
                    self.step_hook(outs)
                if outs:
                    self._deliver(outs)
        except Exception as e:  # engine failure: fail every waiter, mark unhealthy
            self.dead_traceback = traceback.format_exc()
            self.dead = f"{type(e).__name__}: {e}"
            print("[engine] step loop died:\n" + self.dead_traceback, flush=True)
            for q in list(self.queues.values()):
                self.loop.call_soon_threadsafe(q.put_nowait, EngineDeadError(self.dead))

    async def generate(self, prompt, params: SamplingParams, req_id: str,
                       prompt_ids: Optional[list] = None, stream: bool = False,
                       kv_transfer_params: Optional[dict] = None,
                       traceparent: Optional[str] = None) -> AsyncIterator[RequestOutput]:
        if self.dead is not None:
            raise EngineDeadError(self.dead)
        q: asyncio.Queue = asyncio.Queue()
        self.queues[req_id] = q
        try:
            if kv_transfer_params and "transfer_id" in kv_transfer_params:
                first = await self._pull_remote_kv(req_id, params, stream, kv_transfer_params)
                if first is not None:  # first token already ended the request
                    yield first
                    return
            else:
                self.engine.add_request(req_id, prompt, params, prompt_ids=prompt_ids,
                                        stream=stream, kv_transfer_params=kv_transfer_params,
                                        traceparent=traceparent)
            self._wake.set()
            while True:
                o = await q.get()
                if isinstance(o, Exception):
                    raise o
                yield o
                if o.finished:
                    return
        finally:
            self.queues.pop(req_id, None)
            if req_id in self.engine.by_name:  # client went away: free its KV blocks
                self.engine.abort_request(req_id)

    async def _pull_remote_kv(self, req_id: str, params: SamplingParams, stream: bool,
                              kvp: dict) -> Optional[RequestOutput]:
        """P/D decode side: reserve blocks, have the prefill server push the request's KV to
        our rank (batched with other pulls queued at the same moment), receive it over RCCL,
        then let the engine decode.  Every exit path that does not consume the prefill's held
        KV releases it there (/kv/release), so the prefill pod never leaks blocks."""
        eng = self.engine
        prompt_ids = [int(t) for t in kvp["prompt_token_ids"]]
        first = int(kvp["first_token"])
        sp = params.normalized()
        if (not sp.ignore_eos and first == eng.mcfg.eos_id) or sp.max_tokens <= 1:
            # the first token already ends the request: the KV is not needed here
            self._release_remote(kvp)
            reason = "stop" if first == eng.mcfg.eos_id else "length"
            text = "" if reason == "stop" else eng.tokenizer.decode([first])
            return RequestOutput(req_id, prompt_ids, [first], [first], text, text, True,
                                 reason)
        if self.kv_agent is None:
            self._release_remote(kvp)
            raise RuntimeError("this server has no KV-transfer agent (start with --kv-role decode)")
        group = kvp.get("group")
        if group is not None and self.pd_group is not None and group != self.pd_group:
            # prefill of another RCCL group: its send could never pair with our recv
            self._release_remote(kvp)
            raise KVTransferError(f"P/D group mismatch: prefill {group} vs decode "
                                  f"{self.pd_group}")
        if self.puller is None:
            self.puller = KVPuller(self)
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self.puller.submit(PullJob(req_id, prompt_ids, first, params, stream, kvp, fut, loop))
        try:
            await fut
        except (OSError, ValueError, KeyError, RuntimeError, TimeoutError) as e:
            raise KVTransferError(f"KV transfer from {kvp.get('remote_url')} failed: {e}") from e
        if stream:  # the first token was produced remotely: deliver it first
            t = eng.tokenizer.decode_token(first)
            self.queues[req_id].put_nowait(RequestOutput(req_id, prompt_ids, [first], [first],
                                                         t, t, False, None))
        return None

    def peer_id(self) -> str:
        import socket

        return f"{socket.gethostname()}-{os.getpid()}"

    def pair_agent(self, url: str, timeout_s: float = 120.0):
        """Two-pod P/D (decode side): the KV channel to the prefill server at `url`, formed on
        first use by POST /kv/hello and a two-rank group rendezvous at the prefill server's
        TCPStore (the URL's host); a broken one is dropped and re-formed at a new generation."""
        from urllib.parse import urlparse

        from ..parallel.kv_transfer import connect_pair, pair_backend

        with self._pair_lock:
            ag = self.pair_agents.get(url)
            if ag is not None and ag.broken is None:
                return ag
            if ag is not None:
                ag.close()
                self.pair_agents.pop(url, None)
            self._pair_gen += 1
            gen = self._pair_gen
            backend = pair_backend(self.kv_agent.kv)
            body = json.dumps({"peer": self.peer_id(), "generation": gen, "backend": backend,
                               "group": self.pd_group}).encode()
            req = urllib.request.Request(url.rstrip("/") + "/kv/hello", data=body,
                                         headers={"Content-Type": "application/json"})
            with urllib.request.urlopen(req, timeout=30) as r:
                meta = json.loads(r.read())
            ag = connect_pair(self.kv_agent.segs, urlparse(url).hostname, meta["store_port"],
                              meta["prefix"], backend, timeout_s=timeout_s)
            ag.generation = gen
            self.pair_agents[url] = ag
            print(f"[pd] KV channel to {url} formed (generation {gen}, {backend})", flush=True)
            return ag

    def rebuild_channel(self, url: str, timeout_s: float = 120.0) -> bool:
        """Decode side: move both ends of the KV channel to a fresh process group (the next
        generation).  The prefill server joins through POST /kv/reset while this process's
        agent joins here; both block in the group rendezvous until the other arrives."""
        agent = self.kv_agent
        gen = agent.generation + 1
        res: dict = {}

        def remote():
            try:
                body = json.dumps({"generation": gen}).encode()
                req = urllib.request.Request(url.rstrip("/") + "/kv/reset", data=body,
                                             headers={"Content-Type": "application/json"})
                with urllib.request.urlopen(req, timeout=timeout_s) as r:
                    res["remote"] = json.loads(r.read())
            except Exception as e:
                res["error"] = e

        th = threading.Thread(target=remote, name="kv-reset", daemon=True)
        th.start()
        try:
            agent.reset(gen, timeout_s=timeout_s)
        except Exception as e:
            print(f"[pd] KV channel reset to generation {gen} failed: {e}", flush=True)
            return False
        th.join(timeout_s)
        ok = agent.generation == gen and "error" not in res
        print(f"[pd] KV channel rebuilt: generation {gen} ({'ok' if ok else res})", flush=True)
        return ok

    @staticmethod
    def _release_remote(kvp: dict) -> None:
        """Best effort: tell the prefill server to free the held KV of this transfer."""
        url = kvp.get("remote_url")
        if not url or "transfer_id" not in kvp:
            return

        def go():
            try:
                body = json.dumps({"transfer_ids": [int(kvp["transfer_id"])]}).encode()
                req = urllib.request.Request(url.rstrip("/") + "/kv/release", data=body,
                                             headers={"Content-Type": "application/json"})
                urllib.request.urlopen(req, timeout=10).read()
            except Exception as e:  # the prefill side's TTL frees it eventually
                print(f"[pd] /kv/release to {url} failed: {e}", flush=True)

        threading.Thread(target=go, name="kv-release", daemon=True).start()

    async def abort(self, req_id: str) -> None:
        self.engine.abort_request(req_id)
