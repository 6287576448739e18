"""OpenAI-compatible HTTP server for one engine replica (the llm-d "model server").

Routes (contract observed by the reference: llm-d-test.yaml:32-78 and the OTel scrape
of /metrics on :8000, otel-observability-setup.yaml:337-391):
  GET  /v1/models            -> model list (id = served model name, e.g. Qwen/Qwen3-0.6B)
  POST /v1/completions       -> text completion (stream / non-stream, OpenAI schema)
  POST /v1/chat/completions  -> chat completion through a Jinja chat template
  POST /tokenize, /detokenize
  GET  /health, /ready, /version, /metrics (Prometheus text)
"""
from __future__ import annotations

import argparse
import asyncio
import contextlib
import json
import os
import time
import uuid
from typing import Any, Optional

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse

from .. import __version__
from ..engine.config import EngineConfig, SamplingParams
from ..utils import chat_template, tracing
from .async_engine import AsyncEngine, EngineDeadError


def _err(status: int, msg: str, typ: str = "invalid_request_error") -> JSONResponse:
    return JSONResponse({"object": "error", "message": msg, "type": typ, "code": status},
                        status_code=status)


def _sampling_from(body: dict, default_max: int = 16) -> SamplingParams:
    stop = body.get("stop") or []
    if isinstance(stop, str):
        stop = [stop]
    max_tokens = body.get("max_tokens", body.get("max_completion_tokens"))
    return SamplingParams(
        max_tokens=int(max_tokens) if max_tokens is not None else default_max,
        temperature=float(body.get("temperature", 1.0) if body.get("temperature") is not None else 1.0),
        top_p=float(body.get("top_p", 1.0) if body.get("top_p") is not None else 1.0),
        top_k=int(body.get("top_k", 0) or 0),
        min_tokens=int(body.get("min_tokens", 0) or 0),
        seed=body.get("seed"),
        stop=list(stop),
        stop_token_ids=list(body.get("stop_token_ids") or []),
        ignore_eos=bool(body.get("ignore_eos", False)),
        n=int(body.get("n", 1) or 1),
        presence_penalty=float(body.get("presence_penalty") or 0.0),
        frequency_penalty=float(body.get("frequency_penalty") or 0.0),
        repetition_penalty=float(body.get("repetition_penalty") or 1.0),
        logprobs=_logprobs_of(body),
    )


def _logprobs_of(body: dict) -> Optional[int]:
    """completions: "logprobs": int; chat: "logprobs": bool (+ "top_logprobs": int).  The
    sampled token's log-prob plus, for N > 0, the N most likely alternatives per token."""
    lp = body.get("logprobs")
    if lp is None or lp is False:
        return None
    if lp is True:
        return int(body.get("top_logprobs") or 0)
    return int(lp)


def _completion_logprobs(tokenizer, ids: list, lps: list, offset0: int = 0,
                         top: Optional[list] = None) -> dict:
    toks = [tokenizer.decode_token(t) for t in ids]
    offs, o = [], offset0
    for t in toks:
        offs.append(o)
        o += len(t)
    if top:
        tops = [{tokenizer.decode_token(a): v for a, v in alts} for alts in top]
    else:
        tops = [{t: lp} for t, lp in zip(toks, lps)]
    return {"tokens": toks, "token_logprobs": lps, "top_logprobs": tops, "text_offset": offs}


def _chat_logprobs(tokenizer, ids: list, lps: list, top: Optional[list] = None) -> dict:
    def entry(tid, lp):
        s = tokenizer.decode_token(tid)
        return {"token": s, "logprob": lp, "bytes": list(s.encode("utf-8"))}

    out = []
    for i, (t, lp) in enumerate(zip(ids, lps)):
        e = entry(t, lp)
        alts = top[i] if top and i < len(top) else [(t, lp)]
        e["top_logprobs"] = [entry(a, v) for a, v in alts]
        out.append(e)
    return {"content": out}


def _prompts_of(prompt) -> list:
    """OpenAI 'prompt' may be str | list[str] | list[int] | list[list[int]]."""
    if isinstance(prompt, str):
        return [prompt]
    if isinstance(prompt, list) and prompt and all(isinstance(x, int) for x in prompt):
        return [prompt]
    if isinstance(prompt, list):
        return list(prompt)
    raise ValueError("prompt must be a string, a list of strings or token ids")


class OpenAIServer:
    def __init__(self, aengine: AsyncEngine, served_name: str, chat_tmpl: Optional[str],
                 max_model_len: int):
        self.ae = aengine
        self.name = served_name
        self.template = chat_template.load_template(chat_tmpl)
        self.max_model_len = max_model_len
        self.created = int(time.time())
        self._dropped_push = False  # fault injection (AKAP_FAULT_KV_PUSH=drop_once)
        self._ipc_meta = None  # hipIpc export of this engine's KV cache (made on first lease)
        # transfer id -> blocks handed out by /kv/lease (owned by the lease until /kv/done or
        # a /kv/push fallback): the server's own record, never the client's block list
        self._leases: dict[int, list[int]] = {}
        self.app = self._build()

    # ------------------------------------------------------------------ helpers
    def _model_ok(self, body: dict) -> Optional[JSONResponse]:
        m = body.get("model")
        if m is not None and m != self.name:
            return _err(404, f"The model `{m}` does not exist.", "NotFoundError")
        return None

    async def _collect(self, prompt, sp: SamplingParams, rid: str, prompt_ids=None, kvp=None,
                       tp=None):
        final = None
        async for o in self.ae.generate(prompt, sp, rid, prompt_ids=prompt_ids, stream=False,
                                        kv_transfer_params=kvp, traceparent=tp):
            final = o
        return final

    def _pd_guard(self, body: dict, n_jobs: int) -> Optional[JSONResponse]:
        """P/D decode: one pulled transfer feeds exactly one sequence."""
        kvp = body.get("kv_transfer_params")
        if kvp and "transfer_id" in kvp and n_jobs != 1:
            AsyncEngine._release_remote(kvp)
            return _err(400, "P/D decode takes a single prompt with n=1")
        return None

    def _attach_kvp(self, resp: dict, outs: list) -> None:
        """P/D prefill: one decode engine pulls ONE transfer per response (the gateway sends
        n=1 single-prompt requests through P/D); the held KV of any further choice / prompt
        is freed now instead of waiting for its TTL."""
        kvps = [o.kv_transfer_params for o in outs if o is not None and o.kv_transfer_params]
        if not kvps:
            return
        resp["kv_transfer_params"] = kvps[0]
        for k in kvps[1:]:
            self.ae.engine.free_held(int(k["transfer_id"]))

    # ------------------------------------------------------------------ routes
    def _build(self) -> FastAPI:
        @contextlib.asynccontextmanager
        async def lifespan(_app):
            if not self.ae._thread.is_alive():
                self.ae.start(asyncio.get_running_loop())
            yield
            self.ae.stop()

        app = FastAPI(title="akap MI355X OpenAI server", version=__version__, lifespan=lifespan)
        eng = self.ae.engine

        @app.get("/health")
        async def health():
            if not self.ae.healthy:
                return _err(503, "engine dead", "ServiceUnavailable")
            ag = self.ae.kv_agent
            if ag is None:
                return {"status": "ok"}
            # P/D: a broken KV channel is rebuilt by the decode side (/kv/reset); until then
            # the gateway's picker keeps this pair out of P/D routing
            broken = getattr(ag, "broken", None)
            return {"status": "ok", "kv_channel": "broken" if broken else "ok",
                    "kv_generation": getattr(ag, "generation", 0)}

        @app.get("/ready")
        async def ready():
            return await health()

        @app.get("/version")
        async def version():
            return {"version": __version__, "backend": "akap-mi355x", "model": self.name}

        @app.get("/metrics")
        async def metrics():
            eng._update_gauges()
            body = eng.metrics.render()
            # this process's telemetry (kernel-stats windows, GPU counters) and, on rank 0 of a
            # multi-process TP engine, every follower rank's (exporter/rank_metrics.py)
            extra = [t() for t in getattr(self.ae, "telemetry", [])]
            tag = getattr(self.ae, "rank_metrics_tag", None)
            if tag:
                from ..exporter import rank_metrics

                extra += rank_metrics.read_peers(tag)
            if extra:
                from ..exporter import rank_metrics

                body = body.rstrip("\n") + "\n" + rank_metrics.merge(extra)
            return PlainTextResponse(body, media_type="text/plain; version=0.0.4; charset=utf-8")

        @app.get("/v1/models")
        async def models():
            return {"object": "list", "data": [{
                "id": self.name, "object": "model", "created": self.created,
                "owned_by": "akap", "root": self.name, "parent": None,
                "max_model_len": self.max_model_len}]}

        @app.post("/tokenize")
        async def tokenize(req: Request):
            body = await req.json()
            if "messages" in body:
                text = chat_template.render(body["messages"], self.template,
                                            body.get("add_generation_prompt", True))
            else:
                text = body.get("prompt", "")
            toks = eng.tokenizer.encode(text)
            return {"tokens": toks, "count": len(toks), "max_model_len": self.max_model_len}

        @app.post("/detokenize")
        async def detokenize(req: Request):
            body = await req.json()
            return {"prompt": eng.tokenizer.decode(body.get("tokens", []))}

        @app.post("/kv/push")
        async def kv_push(req: Request):
            """P/D prefill side: send the held KV of one or more transfers to the decode rank
            as ONE packed RCCL send (the decode side posts one matching recv)."""
            body = await req.json()
            if self.ae.kv_agent is None:
                return _err(400, "not a P/D prefill server")
            grp = body.get("group")
            if grp is not None and self.ae.pd_group is not None and grp != self.ae.pd_group:
                return _err(409, f"P/D group mismatch: decode {grp} vs prefill "
                                 f"{self.ae.pd_group}", "Conflict")
            agent = self.ae.kv_agent
            if body.get("peer") is not None:  # two-pod bootstrap: this peer's pair channel
                host = getattr(self.ae, "pair_host", None)
                agent = host.agent(str(body["peer"])) if host is not None else None
                if agent is None:
                    return _err(409, f"no KV channel to peer {body['peer']} (POST /kv/hello)",
                                "KVChannelBroken")
            if getattr(agent, "broken", None) is not None:
                # the decode side rebuilds the channel (/kv/reset, or a new /kv/hello) and
                # retries later requests
                return _err(503, f"KV channel broken: {agent.broken}", "KVChannelBroken")
            tids = [int(t) for t in (body.get("transfer_ids") or [body["transfer_id"]])]
            if body.get("leased_blocks") is not None:
                # the decode side leased these transfers for a hipIpc pull and could not map
                # this cache in time: the lease already owns the blocks (until finish_transfer).
                # The blocks come from this server's lease record; the client's list must
                # match it exactly (a stale or forged list would ship other requests' KV or
                # index past the cache)
                claimed = body["leased_blocks"]
                if not isinstance(claimed, list) or len(claimed) != len(tids):
                    return _err(400, "leased_blocks: one block list per transfer id")
                unknown = [t for t in tids if t not in self._leases]
                if unknown:
                    return _err(404, f"no lease for transfer(s) {unknown}")
                try:
                    claimed = [[int(b) for b in bl] for bl in claimed]
                except (TypeError, ValueError):
                    return _err(400, "leased_blocks: integer block ids")
                per = [self._leases[t] for t in tids]
                if claimed != per:
                    return _err(409, "leased_blocks do not match this server's leases",
                                "Conflict")
                for t in tids:
                    self._leases.pop(t, None)
            else:
                per = [eng.held_blocks(t) for t in tids]
                missing = [t for t, b in zip(tids, per) if not b]
                if missing:
                    return _err(404, f"no held KV for transfer(s) {missing}")
                # from here the blocks are owned by the send (not the TTL sweep, not
                # /kv/release) until its completion frees them
                per = [eng.take_held(t) for t in tids]
                if any(not b for b in per):  # expired between the check and the take
                    for t in tids:
                        eng.finish_transfer(t)
                    return _err(404, f"held KV for transfer(s) {tids} expired")
            blocks = [b for bl in per for b in bl]
            fault = os.environ.get("AKAP_FAULT_KV_PUSH")
            if fault == "drop" or (fault == "drop_once" and not self._dropped_push):
                self._dropped_push = True
                # fault injection (tests): acknowledge the push, then "die" before sending --
                # the decode side's bounded recv must fail the request, not hang
                for t in tids:
                    eng.finish_transfer(t)
                return {"ok": True, "num_blocks": [len(b) for b in per]
                        if "transfer_ids" in body else len(per[0])}

            def done(ts=tuple(tids)):
                for t in ts:
                    eng.finish_transfer(t)

            agent.send_blocks(blocks, int(body["dst_rank"]), on_done=done)
            nb = [len(b) for b in per]
            return {"ok": True, "num_blocks": nb if "transfer_ids" in body else nb[0]}

        @app.post("/kv/hello")
        async def kv_hello(req: Request):
            """Two-pod P/D (prefill side): open a two-rank KV channel for a decode server
            started on its own -- returns the TCPStore port and the group prefix it joins as
            rank 1 while this server joins as rank 0 (in the background)."""
            body = await req.json()
            host = getattr(self.ae, "pair_host", None)
            if host is None:
                return _err(400, "not a two-pod (--pd-bootstrap http) prefill server")
            grp = body.get("group")
            if grp is not None and grp != self.ae.pd_group:
                return _err(409, f"P/D group mismatch: decode {grp} vs prefill "
                                 f"{self.ae.pd_group}", "Conflict")
            prefix = host.accept(str(body["peer"]), int(body.get("generation", 0)),
                                 str(body.get("backend", "gloo")))
            return {"ok": True, "store_port": host.port, "prefix": prefix}

        @app.post("/kv/lease")
        async def kv_lease(req: Request):
            """P/D prefill side, hipIpc transport: lease the held KV of one or more transfers
            to the decode engine, which pulls the blocks itself out of this engine's cache
            (mapped once from `ipc`); the blocks stay owned by the lease until /kv/done."""
            body = await req.json()
            ag = self.ae.kv_agent
            if ag is None or not getattr(ag, "is_gpu", False):
                return _err(400, "not a GPU P/D prefill server")
            tids = [int(t) for t in body["transfer_ids"]]
            per = [eng.held_blocks(t) for t in tids]
            missing = [t for t, b in zip(tids, per) if not b]
            if missing:
                return _err(404, f"no held KV for transfer(s) {missing}")
            per = [eng.take_held(t) for t in tids]
            if any(not b for b in per):  # expired between the check and the take
                for t in tids:
                    eng.finish_transfer(t)
                return _err(404, f"held KV for transfer(s) {tids} expired")
            if self._ipc_meta is None:
                self._ipc_meta = ag.ipc_meta()
            for t, bl in zip(tids, per):
                self._leases[t] = [int(b) for b in bl]
            return {"ok": True, "blocks": [[int(b) for b in bl] for bl in per],
                    "ipc": self._ipc_meta}

        @app.post("/kv/done")
        async def kv_done(req: Request):
            """P/D prefill side: the decode engine finished pulling (or gave up on) these
            leased transfers: free their blocks."""
            body = await req.json()
            for t in body["transfer_ids"]:
                self._leases.pop(int(t), None)
                eng.finish_transfer(int(t))
            return {"ok": True}

        @app.post("/kv/reset")
        async def kv_reset(req: Request):
            """P/D: rebuild the KV-transfer channel (a fresh process group over the same ranks)
            at the given generation.  The decode side calls this while resetting its own
            agent; both calls return once the new group is formed."""
            body = await req.json()
            if self.ae.kv_agent is None:
                return _err(400, "not a P/D server")
            gen = int(body["generation"])
            try:
                moved = await asyncio.get_running_loop().run_in_executor(
                    None, self.ae.kv_agent.reset, gen)
            except Exception as e:  # rendezvous timed out: the channel stays broken
                return _err(503, f"KV channel reset to generation {gen} failed: {e}",
                            "ServiceUnavailable")
            return {"ok": True, "generation": self.ae.kv_agent.generation, "moved": moved}

        @app.post("/kv/release")
        async def kv_release(req: Request):
            """P/D prefill side: the decode side will not pull these transfers (first token
            ended the request, decode failure, retry): free their held KV now."""
            body = await req.json()
            tids = [int(t) for t in (body.get("transfer_ids") or [body["transfer_id"]])]
            for t in tids:
                self._leases.pop(t, None)
                eng.free_held(t)
            return {"ok": True, "released": len(tids)}

        @app.post("/v1/completions")
        async def completions(req: Request):
            try:
                body = await req.json()
            except Exception:
                return _err(400, "invalid JSON body")
            bad = self._model_ok(body)
            if bad:
                return bad
            try:
                sp = _sampling_from(body)
                prompts = _prompts_of(body.get("prompt", ""))
            except (ValueError, TypeError) as e:
                return _err(400, str(e))
            bad = self._pd_guard(body, len(prompts) * sp.n)
            if bad:
                return bad
            cid = f"cmpl-{uuid.uuid4().hex}"
            created = int(time.time())
            tp = req.headers.get("traceparent")
            if body.get("stream"):
                # every (prompt, choice) streams as its own choice index i * n + j
                return StreamingResponse(self._stream_completion(cid, created, prompts, sp,
                                                                 body, tp),
                                         media_type="text/event-stream")
            try:
                jobs = []
                for i, p in enumerate(prompts):
                    for j in range(sp.n):
                        pid = p if isinstance(p, list) else None
                        jobs.append(self._collect(p if isinstance(p, str) else None, sp,
                                                  f"{cid}-{i}-{j}", prompt_ids=pid,
                                                  kvp=body.get("kv_transfer_params"), tp=tp))
                outs = await asyncio.gather(*jobs)
            except EngineDeadError as e:
                return _err(500, "engine failure: " + str(e)[:200], "InternalServerError")
            except ValueError as e:
                return _err(400, str(e))
            except RuntimeError as e:
                return _err(503, str(e), "ServiceUnavailable")
            choices, ptok, ctok = [], 0, 0
            for k, o in enumerate(outs):
                text = o.text
                if body.get("echo") and isinstance(prompts[k // sp.n], str):
                    text = prompts[k // sp.n] + text
                lpd = None
                if sp.logprobs is not None and o.logprobs is not None:
                    lpd = _completion_logprobs(self.ae.engine.tokenizer, o.output_ids,
                                               o.logprobs, top=o.top_logprobs)
                choices.append({"index": k, "text": text, "logprobs": lpd,
                                "finish_reason": o.finish_reason, "stop_reason": None})
                ctok += len(o.output_ids)
                if k % sp.n == 0:
                    ptok += len(o.prompt_ids)
            resp = {"id": cid, "object": "text_completion", "created": created,
                    "model": self.name, "choices": choices,
                    "usage": {"prompt_tokens": ptok, "completion_tokens": ctok,
                              "total_tokens": ptok + ctok}}
            self._attach_kvp(resp, outs)
            return resp

        @app.post("/v1/chat/completions")
        async def chat(req: Request):
            try:
                body = await req.json()
            except Exception:
                return _err(400, "invalid JSON body")
            bad = self._model_ok(body)
            if bad:
                return bad
            msgs = body.get("messages")
            if not isinstance(msgs, list) or not msgs:
                return _err(400, "messages must be a non-empty list")
            tmpl = self.template
            if body.get("chat_template"):
                try:
                    tmpl = chat_template.load_template(body["chat_template"])
                except ValueError as e:
                    return _err(400, str(e))
            try:
                prompt = chat_template.render(msgs, tmpl, body.get("add_generation_prompt", True))
                sp = _sampling_from(body, default_max=max(16, self.max_model_len // 4))
            except Exception as e:
                return _err(400, f"chat template error: {e}")
            bad = self._pd_guard(body, sp.n)
            if bad:
                return bad
            cid = f"chatcmpl-{uuid.uuid4().hex}"
            created = int(time.time())
            tp = req.headers.get("traceparent")
            if body.get("stream"):
                return StreamingResponse(self._stream_chat(cid, created, prompt, sp, body, tp),
                                         media_type="text/event-stream")
            try:
                outs = await asyncio.gather(*[self._collect(prompt, sp, f"{cid}-{j}",
                                                            kvp=body.get("kv_transfer_params"),
                                                            tp=tp)
                                              for j in range(sp.n)])
            except EngineDeadError as e:
                return _err(500, "engine failure: " + str(e)[:200], "InternalServerError")
            except ValueError as e:
                return _err(400, str(e))
            except RuntimeError as e:
                return _err(503, str(e), "ServiceUnavailable")
            tok = self.ae.engine.tokenizer
            choices = [{"index": j, "message": {"role": "assistant", "content": o.text},
                        "logprobs": (_chat_logprobs(tok, o.output_ids, o.logprobs,
                                                    o.top_logprobs)
                                     if sp.logprobs is not None and o.logprobs is not None
                                     else None),
                        "finish_reason": o.finish_reason}
                       for j, o in enumerate(outs)]
            ptok = len(outs[0].prompt_ids)
            ctok = sum(len(o.output_ids) for o in outs)
            resp = {"id": cid, "object": "chat.completion", "created": created,
                    "model": self.name, "choices": choices,
                    "usage": {"prompt_tokens": ptok, "completion_tokens": ctok,
                              "total_tokens": ptok + ctok}}
            self._attach_kvp(resp, outs)
            return resp

        return app

    # ------------------------------------------------------------------ SSE
    @staticmethod
    async def _merged(gens):
        """Interleave several engine streams as (choice index, output) in arrival order."""
        if len(gens) == 1:  # the common single-choice stream: no task/queue hop
            async for o in gens[0]:
                yield 0, o
            return
        q: asyncio.Queue = asyncio.Queue()

        async def pump(k, g):
            try:
                async for o in g:
                    await q.put((k, o))
            except Exception as e:  # noqa: BLE001 -- re-raised in the consumer
                await q.put((k, e))
            await q.put((k, None))

        tasks = [asyncio.create_task(pump(k, g)) for k, g in enumerate(gens)]
        live = len(tasks)
        try:
            while live:
                k, o = await q.get()
                if o is None:
                    live -= 1
                elif isinstance(o, Exception):
                    raise o
                else:
                    yield k, o
        finally:
            for t in tasks:
                t.cancel()

    async def _stream_completion(self, cid, created, prompts, sp, body, tp=None):
        gens = []
        for i, p in enumerate(prompts):
            for j in range(sp.n):
                gens.append(self.ae.generate(
                    p if isinstance(p, str) else None, sp,
                    cid if len(prompts) * sp.n == 1 else f"{cid}-{i}-{j}",
                    prompt_ids=p if isinstance(p, list) else None, stream=True,
                    kv_transfer_params=body.get("kv_transfer_params"), traceparent=tp))
        n_out, n_prompt = {}, {}
        try:
            async for k, o in self._merged(gens):
                n_out[k], n_prompt[k] = len(o.output_ids), len(o.prompt_ids)
                chunk = {"id": cid, "object": "text_completion", "created": created,
                         "model": self.name, "choices": [{
                             "index": k, "text": o.delta_text, "logprobs": None,
                             "finish_reason": o.finish_reason if o.finished else None}]}
                yield f"data: {json.dumps(chunk)}\n\n"
        except Exception as e:  # surface errors in-band, as vLLM does
            yield f"data: {json.dumps({'error': {'message': str(e)[:300]}})}\n\n"
        if (body.get("stream_options") or {}).get("include_usage"):
            pt = sum(v for k, v in n_prompt.items() if k % sp.n == 0)
            ct = sum(n_out.values())
            u = {"id": cid, "object": "text_completion", "created": created, "model": self.name,
                 "choices": [], "usage": {"prompt_tokens": pt, "completion_tokens": ct,
                                          "total_tokens": pt + ct}}
            yield f"data: {json.dumps(u)}\n\n"
        yield "data: [DONE]\n\n"

    async def _stream_chat(self, cid, created, prompt, sp, body, tp=None):
        for j in range(sp.n):
            first = {"id": cid, "object": "chat.completion.chunk", "created": created,
                     "model": self.name, "choices": [{"index": j, "delta": {
                         "role": "assistant", "content": ""}, "finish_reason": None}]}
            yield f"data: {json.dumps(first)}\n\n"
        gens = [self.ae.generate(prompt, sp, cid if sp.n == 1 else f"{cid}-{j}", stream=True,
                                 kv_transfer_params=body.get("kv_transfer_params"),
                                 traceparent=tp) for j in range(sp.n)]
        n_out, n_prompt = {}, 0
        try:
            async for k, o in self._merged(gens):
                n_out[k], n_prompt = len(o.output_ids), len(o.prompt_ids)
                chunk = {"id": cid, "object": "chat.completion.chunk", "created": created,
                         "model": self.name, "choices": [{
                             "index": k, "delta": {"content": o.delta_text} if o.delta_text else {},
                             "finish_reason": o.finish_reason if o.finished else None}]}
                yield f"data: {json.dumps(chunk)}\n\n"
        except Exception as e:
            yield f"data: {json.dumps({'error': {'message': str(e)[:300]}})}\n\n"
        if (body.get("stream_options") or {}).get("include_usage"):
            ct = sum(n_out.values())
            u = {"id": cid, "object": "chat.completion.chunk", "created": created,
                 "model": self.name, "choices": [],
                 "usage": {"prompt_tokens": n_prompt, "completion_tokens": ct,
                           "total_tokens": n_prompt + ct}}
            yield f"data: {json.dumps(u)}\n\n"
        yield "data: [DONE]\n\n"


def make_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser("akap-serve", description="MI355X OpenAI-compatible server")
    ap.add_argument("--model", default=os.environ.get("AKAP_MODEL", "qwen3-0.6b"))
    ap.add_argument("--served-model-name", default=None)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-num-batched-tokens", type=int, default=16384)
    ap.add_argument("--block-size", type=int, default=32)
    ap.add_argument("--gpu-memory-utilization", type=float, default=0.90)
    ap.add_argument("--num-gpu-blocks", type=int, default=None)
    ap.add_argument("--tensor-parallel-size", "-tp", type=int, default=1)
    ap.add_argument("--enforce-eager", action="store_true")
    ap.add_argument("--no-enable-prefix-caching", action="store_true")
    ap.add_argument("--chat-template", default=None)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--load-format", default="random", choices=["random", "safetensors"])
    ap.add_argument("--weights-path", default=None)
    ap.add_argument("--kv-role", default="both", choices=["both", "prefill", "decode"])
    ap.add_argument("--pd-bootstrap", default=os.environ.get("AKAP_PD_BOOTSTRAP", "launcher"),
                    choices=["launcher", "http"],
                    help="P/D roles: launcher = every prefill/decode rank of one torch.distributed "
                         "job (server/pd_launch.py, one pod); http = independently started "
                         "servers (separate prefill / decode Deployments): the decode server "
                         "bootstraps a KV channel per prefill peer over HTTP (/kv/hello -> "
                         "the prefill server's TCPStore), the hipIpc pull needs none")
    ap.add_argument("--kv-store-port", type=int,
                    default=int(os.environ.get("AKAP_KV_STORE_PORT", "29710")),
                    help="--pd-bootstrap http, prefill role: TCPStore port of the pair channels")
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8", "fp8_e4m3"],
                    help="fp8: OCP e4m3 KV cache (half the bytes; decode attention streams "
                         "half as much)")
    ap.add_argument("--otlp-traces-endpoint", default=None,
                    help="OTLP/HTTP collector (e.g. http://otel-collector:4318); also read "
                         "from OTEL_EXPORTER_OTLP_TRACES_ENDPOINT")
    ap.add_argument("--kernel-stats-interval", type=float, default=0.0,
                    help="seconds between in-process GPU kernel-stats windows served as "
                         "akap_kernel_* on /metrics (torch.profiler; 0 = off, the rocprofv3 "
                         "sidecar then provides them)")
    ap.add_argument("--kernel-stats-window-ms", type=int, default=1000)
    ap.add_argument("--pmc-interval", type=float, default=0.0,
                    help="seconds between GPU hardware-counter reads served as akap_gpu_pmc_* "
                         "on /metrics (0 = off; needs ROCP_TOOL_LIBRARIES=<libakap_pmc.so> in "
                         "the environment at process start)")
    return ap


def engine_config_from_args(a) -> EngineConfig:
    return EngineConfig(
        model=a.model, served_model_name=a.served_model_name, max_model_len=a.max_model_len,
        max_num_seqs=a.max_num_seqs, max_num_batched_tokens=a.max_num_batched_tokens,
        block_size=a.block_size, gpu_memory_utilization=a.gpu_memory_utilization,
        num_gpu_blocks=a.num_gpu_blocks, enable_prefix_caching=not a.no_enable_prefix_caching,
        enforce_eager=a.enforce_eager, tensor_parallel_size=a.tensor_parallel_size, seed=a.seed,
        device=a.device, load_format=a.load_format, weights_path=a.weights_path,
        chat_template=a.chat_template, kv_role=a.kv_role, kv_cache_dtype=a.kv_cache_dtype)


def pd_group_id() -> str:
    """Identity of this process's P/D transfer group (the torch.distributed group shared by a
    prefill and a decode rank): AKAP_PD_GROUP, else host + rendezvous port.  The prefill side
    stamps it into kv_transfer_params; the decode side refuses a transfer from another group
    (its RCCL send could never pair with our recv) instead of hanging."""
    g = os.environ.get("AKAP_PD_GROUP")
    if g:
        return g
    import socket

    return f"{socket.gethostname()}:{os.environ.get('MASTER_ADDR', '')}:" \
           f"{os.environ.get('MASTER_PORT', '')}"


def make_telemetry(a, labels: dict) -> list:
    """This process's in-process telemetry providers (text callables for /metrics): kernel-stats
    windows (--kernel-stats-interval) and GPU hardware counters (--pmc-interval), labelled with
    `labels` (the TP rank in multi-process engines)."""
    from ..exporter import rank_metrics

    out = []
    if a.kernel_stats_interval > 0:
        from ..exporter.inprocess_profiler import InProcessKernelProfiler

        kp = InProcessKernelProfiler(a.kernel_stats_window_ms, a.kernel_stats_interval).start()
        out.append(lambda: rank_metrics.add_labels(kp.text(), labels))
    if a.pmc_interval > 0:
        from ..exporter.pmc_sampler import PMCSampler

        pmc = PMCSampler(a.pmc_interval, labels=labels).start()
        out.append(pmc.text)
    return out


def build_app(ecfg: EngineConfig, engine=None, pd_bootstrap: str = "launcher",
              kv_store_port: int = 29710) -> tuple[FastAPI, AsyncEngine]:
    from ..engine.llm_engine import LLMEngine

    eng = engine or LLMEngine(ecfg)
    ae = AsyncEngine(eng)
    if ecfg.kv_role in ("prefill", "decode"):
        from ..parallel.kv_transfer import KVTransferAgent

        ae.kv_agent = KVTransferAgent(eng.runner.kv_segs)
        ae.pd_bootstrap = pd_bootstrap
        if pd_bootstrap == "http":
            # two-pod P/D: no shared job; every prefill/decode pair is its own two-rank channel
            # (prefill rank 0, decode rank 1), formed on demand; servers of one deployment
            # share AKAP_PD_GROUP (the gateway pairs only inside it)
            ae.pd_group = eng.pd_group = os.environ.get("AKAP_PD_GROUP", "http")
            eng.rank = 0 if ecfg.kv_role == "prefill" else 1
            if ecfg.kv_role == "prefill":
                from ..parallel.kv_transfer import PairHost

                ae.pair_host = PairHost(eng.runner.kv_segs, kv_store_port)
        else:
            ae.pd_group = eng.pd_group = pd_group_id()
        eng.kv_agent = ae.kv_agent
        if ecfg.kv_role == "decode":
            from .async_engine import decode_transport

            # /metrics akap:kv_transport_ipc: 1 while this decode server pulls KV by hipIpc
            # (no prefill peer fell back to p2p) -- the gateway prefers such pairs
            eng.kv_ipc_state = lambda: (decode_transport(ae.kv_agent) == "ipc" and not (
                ae.puller is not None and ae.puller.ipc_fallback))
    srv = OpenAIServer(ae, eng.model_name, ecfg.chat_template, ecfg.max_model_len)
    return srv.app, ae


def main(argv: Optional[list] = None) -> None:
    import uvicorn

    a = make_parser().parse_args(argv)
    ecfg = engine_config_from_args(a)
    tracing.configure(a.otlp_traces_endpoint, service_name=os.environ.get(
        "OTEL_SERVICE_NAME", f"akap-engine-{a.kv_role}"))
    if a.tensor_parallel_size > 1:
        from ..parallel.tp_worker import serve_tp

        serve_tp(ecfg, a.host, a.port, telemetry=lambda labels: make_telemetry(a, labels))
        return
    if a.kv_role != "both" and a.pd_bootstrap == "http" and a.device != "cpu":
        # two-pod P/D: log RCCL's connection transports so the channel probe can report which
        # one the pair channel got (P2P over xGMI vs SHM vs NET sockets)
        from ..parallel.kv_transfer import enable_rccl_transport_log

        enable_rccl_transport_log()
    if a.kv_role != "both" and a.pd_bootstrap == "launcher":
        # P/D: this process is one rank of the prefill/decode KV-transfer group (torchrun)
        from ..parallel.state import init_distributed

        backend = os.environ.get("AKAP_DIST_BACKEND") or ("gloo" if a.device == "cpu" else None)
        init_distributed(tp_size=1, backend=backend)
    app, ae = build_app(ecfg, pd_bootstrap=a.pd_bootstrap, kv_store_port=a.kv_store_port)
    ae.telemetry = make_telemetry(a, {})
    uvicorn.run(app, host=a.host, port=a.port, log_level="info", access_log=False)


if __name__ == "__main__":
    main()
