"""Asyncio front of the engine: one background thread drives LLMEngine.step() while
HTTP handlers await per-request output queues.

The step loop never blocks the event loop (GPU work + the C++ scheduler run in the
engine thread; outputs are handed over with call_soon_threadsafe).  When idle the
thread parks on an Event, so an idle pod burns no CPU.
"""
from __future__ import annotations

import asyncio
import threading
import time
import traceback
from typing import AsyncIterator, Optional

from ..engine.config import SamplingParams
from ..engine.llm_engine import LLMEngine, RequestOutput


class EngineDeadError(RuntimeError):
    pass


class AsyncEngine:
    def __init__(self, engine: LLMEngine, step_hook=None):
        self.engine = engine
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.queues: dict[str, asyncio.Queue] = {}
        self._wake = threading.Event()
        self._stop = False
        self.dead: Optional[str] = None
        self.step_hook = step_hook  # e.g. P/D KV hand-off after prefill
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
        except Exception:  # engine failure: fail every waiter, mark unhealthy
            self.dead = traceback.format_exc()
            for q in list(self.queues.values()):
                self.loop.call_soon_threadsafe(q.put_nowait, EngineDeadError(self.dead))

    async def generate(self, prompt, params: SamplingParams, req_id: str,
                       prompt_ids: Optional[list] = None, stream: bool = False
                       ) -> AsyncIterator[RequestOutput]:
        if self.dead is not None:
            raise EngineDeadError(self.dead)
        q: asyncio.Queue = asyncio.Queue()
        self.queues[req_id] = q
        try:
            self.engine.add_request(req_id, prompt, params, prompt_ids=prompt_ids, stream=stream)
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

    async def abort(self, req_id: str) -> None:
        self.engine.abort_request(req_id)
