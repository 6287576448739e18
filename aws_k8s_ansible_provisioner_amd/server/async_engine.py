"""Asyncio front of the engine: one background thread drives LLMEngine.step() while
HTTP handlers await per-request output queues.

The step loop never blocks the event loop (GPU work + the C++ scheduler run in the
engine thread; outputs are handed over with call_soon_threadsafe).  When idle the
thread parks on an Event, so an idle pod burns no CPU.
"""
from __future__ import annotations

import asyncio
import json
import threading
import urllib.request
import time
import traceback
from typing import AsyncIterator, Optional

from ..engine.config import SamplingParams
from ..engine.llm_engine import LLMEngine, RequestOutput


class EngineDeadError(RuntimeError):
    pass


class KVTransferError(RuntimeError):
    """P/D: the prefill pod could not hand the request's KV over (pod gone, timeout,
    block-count mismatch).  The decode side frees its reserved blocks and fails the
    request; the gateway may retry it monolithically."""


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
        """P/D decode side: reserve blocks, ask the prefill server to push the request's
        KV to our rank, receive it over RCCL, then let the engine decode."""
        eng = self.engine
        prompt_ids = [int(t) for t in kvp["prompt_token_ids"]]
        first = int(kvp["first_token"])
        sp = params.normalized()
        if (not sp.ignore_eos and first == eng.mcfg.eos_id) or sp.max_tokens <= 1:
            reason = "stop" if first == eng.mcfg.eos_id else "length"
            text = "" if reason == "stop" else eng.tokenizer.decode([first])
            return RequestOutput(req_id, prompt_ids, [first], [first], text, text, True,
                                 reason)
        if self.kv_agent is None:
            raise RuntimeError("this server has no KV-transfer agent (start with --kv-role decode)")
        loop = asyncio.get_running_loop()

        def pull():
            iid, blocks = eng.reserve_prefilled(req_id, prompt_ids, first, params, stream)
            if not blocks:
                raise RuntimeError("KV pool exhausted on the decode engine")
            body = json.dumps({"transfer_id": kvp["transfer_id"], "dst_rank": eng.rank}).encode()
            req = urllib.request.Request(kvp["remote_url"].rstrip("/") + "/kv/push", data=body,
                                         headers={"Content-Type": "application/json"})
            with urllib.request.urlopen(req, timeout=60) as r:
                meta = json.loads(r.read())
            if int(meta.get("num_blocks", -1)) != len(blocks):
                raise RuntimeError(f"KV block count mismatch {meta} vs {len(blocks)}")
            self.kv_agent.recv_blocks(blocks, int(kvp["remote_rank"]))
            eng.activate(iid)

        try:
            await loop.run_in_executor(None, pull)
        except (OSError, ValueError, KeyError, RuntimeError) as e:
            raise KVTransferError(f"KV transfer from {kvp.get('remote_url')} failed: {e}") from e
        if stream:  # the first token was produced remotely: deliver it first
            t = eng.tokenizer.decode_token(first)
            self.queues[req_id].put_nowait(RequestOutput(req_id, prompt_ids, [first], [first],
                                                         t, t, False, None))
        return None

    async def abort(self, req_id: str) -> None:
        self.engine.abort_request(req_id)
