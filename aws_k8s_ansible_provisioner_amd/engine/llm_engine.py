"""LLMEngine: request bookkeeping around the C++ scheduler and the model runner.

One engine = one model replica (one GPU, or one TP group where every rank runs the
same step in lock-step: rank 0 schedules and broadcasts the step, see parallel/tp_worker).
"""
from __future__ import annotations

import dataclasses
import gc
import itertools
import os
import threading
import time
from typing import Iterable, Optional, Union

import numpy as np

from .. import _runtime_loader
from ..models.config import ModelConfig, get_config
from ..utils import tracing
from ..utils.metrics import EngineMetrics
from ..utils.tokenizer import get_tokenizer
from .config import EngineConfig, SamplingParams
from .model_runner import ModelRunner

FINISH_REASONS = {0: None, 1: "length", 2: "stop", 3: "abort"}


@dataclasses.dataclass
class RequestState:
    req_id: str
    iid: int
    prompt: Optional[str]
    prompt_ids: list
    params: SamplingParams
    arrival: float
    output_ids: list = dataclasses.field(default_factory=list)
    logprobs: list = dataclasses.field(default_factory=list)
    top_logprobs: list = dataclasses.field(default_factory=list)  # per token: [(id, lp)]
    first_token_time: Optional[float] = None
    last_token_time: Optional[float] = None
    finish_reason: Optional[str] = None
    finished: bool = False
    text: str = ""
    stream: bool = False
    hold_kv: bool = False
    traceparent: Optional[str] = None
    first_scheduled: Optional[float] = None

    def prompt_list(self) -> list:
        """The prompt ids as a list (an int32 array handed to add_request is converted once,
        off the admission path)."""
        if isinstance(self.prompt_ids, np.ndarray):
            self.prompt_ids = self.prompt_ids.tolist()
        return self.prompt_ids


@dataclasses.dataclass
class RequestOutput:
    req_id: str
    prompt_ids: list
    output_ids: list
    new_ids: list
    text: str
    delta_text: str
    finished: bool
    finish_reason: Optional[str]
    ttft: Optional[float] = None
    num_cached_tokens: int = 0
    kv_transfer_params: Optional[dict] = None
    logprobs: Optional[list] = None  # per output token (when the request asked for them)
    top_logprobs: Optional[list] = None  # per output token: [(token id, log-prob)] x N


class LLMEngine:
    def __init__(self, ecfg: EngineConfig, mcfg: Optional[ModelConfig] = None, pstate=None,
                 log=print, runner: Optional[ModelRunner] = None):
        self.ecfg = ecfg
        self.mcfg = mcfg or get_config(ecfg.model)
        self.model_name = ecfg.served_model_name or self.mcfg.hf_id
        self.log = log
        self.runner = runner or ModelRunner(ecfg, self.mcfg, pstate, log=log)
        rt = _runtime_loader.load()
        sc = rt.SchedConfig()
        sc.max_num_seqs = ecfg.max_num_seqs
        sc.max_num_batched_tokens = ecfg.max_num_batched_tokens
        sc.max_model_len = ecfg.max_model_len
        sc.block_size = ecfg.block_size
        sc.gqa_group = self.runner.G
        sc.tile_rows = self.runner.tile_rows
        sc.tile_rows_short = self.runner.tile_rows_short
        sc.eos_id = self.mcfg.eos_id
        sc.max_blocks_per_seq = self.runner.max_blocks
        sc.mixed_batching = ecfg.mixed_batching
        sc.mix_backlog_steps = ecfg.mix_backlog_steps
        sc.max_decode_stall_steps = ecfg.max_decode_stall_steps
        sc.held_kv_ttl_s = ecfg.held_kv_ttl_s
        sc.num_tail_slots = self.runner.num_tail_slots
        self.sched = rt.Scheduler(sc, self.runner.num_blocks, ecfg.enable_prefix_caching)
        self.tokenizer = get_tokenizer(ecfg.weights_path, self.mcfg.vocab_size, self.mcfg.bos_id,
                                       self.mcfg.eos_id)
        self.metrics = EngineMetrics(self.model_name)
        self.reqs: dict[int, RequestState] = {}
        self.by_name: dict[str, int] = {}
        self._ids = itertools.count(1)
        self._lock = threading.Lock()
        self._pending_aborts: list[int] = []
        self.steps = 0
        self.last_prefix = (0, 0)
        self.timers = {"schedule": 0.0, "execute": 0.0, "post": 0.0}
        # execute wall time / step count per step kind (pure prefill, mixed, pure decode)
        self.step_kinds = {k: [0.0, 0] for k in ("prefill", "mixed", "decode")}
        self._n_extra = 0  # live requests that need penalties or log-probs
        self.last_step_mixed = False  # the last step ran decode rows beside prefill chunks
        self.pd_group: Optional[str] = None  # P/D transfer-group id (stamped into kvp)
        self.kv_agent = None  # P/D: the KVTransferAgent (metrics only)
        self.rank = self.runner.ps.rank
        self._inflight = None  # (info, handle) of a launched lookahead decode step
        self.lookahead_steps = 0
        # decode lookahead: single GPU, DP replicas and TP groups (rank 0 broadcasts the
        # lookahead step's header like any other; parallel/tp_worker); not with expert-
        # parallel MoE (an overflowed dispatch re-runs its step, which a queued successor
        # would already have consumed).  AKAP_ASYNC_DECODE=force: also without hipGraphs
        # (CPU protocol tests; the step then runs eagerly inside launch_decode)
        mode = os.environ.get("AKAP_ASYNC_DECODE", "1")
        self._async_decode = (ecfg.async_decode and mode != "0" and
                              ((self.runner.is_gpu and bool(self.runner.graphs))
                               or mode == "force") and not self.runner._ep_moe)
        if ecfg.gc_freeze and os.environ.get("AKAP_GC_FREEZE", "1") != "0":
            # Move everything alive after start-up (model, graphs, torch/extension objects)
            # into the permanent generation: the serving loop allocates ~10^5 small objects
            # per batch of requests (prompt/output id lists), and a full collection that
            # walks the start-up heap stalled a step by ~0.1 s (measured on the CPU path).
            gc.collect()
            gc.freeze()

    # ------------------------------------------------------------------ requests
    def add_request(self, req_id: Optional[str], prompt: Union[str, list, None],
                    params: Optional[SamplingParams] = None,
                    prompt_ids: Optional[list] = None, stream: bool = False,
                    kv_transfer_params: Optional[dict] = None,
                    traceparent: Optional[str] = None) -> str:
        """Queue a request.  stream=True reports every token (server SSE); otherwise the
        engine reports only the first token (TTFT) and the finished output."""
        params = (params or SamplingParams()).normalized()
        return self._add(req_id, prompt, params, prompt_ids, stream, kv_transfer_params,
                         traceparent)

    def _add(self, req_id, prompt, params: SamplingParams, prompt_ids, stream=False,
             kv_transfer_params=None, traceparent=None) -> str:
        """add_request with params already normalized (generate() normalizes once per batch)."""
        if prompt_ids is None:
            if isinstance(prompt, str):
                prompt_ids = self.tokenizer.encode(prompt)
            else:
                prompt_ids = list(prompt or [])
        if isinstance(prompt_ids, np.ndarray):
            # kept as int32 until an output needs the list (RequestState.prompt_list): the
            # scheduler takes the buffer in one copy
            prompt_ids = np.ascontiguousarray(prompt_ids.reshape(-1), dtype=np.int32)
        else:
            prompt_ids = list(map(int, prompt_ids))  # C-level conversion (a 512-id prompt:
            #                                           ~4x faster than a comprehension)
        if not len(prompt_ids):
            prompt_ids = [self.mcfg.bos_id]
        if len(prompt_ids) >= self.ecfg.max_model_len:
            raise ValueError(f"prompt has {len(prompt_ids)} tokens; max_model_len is "
                             f"{self.ecfg.max_model_len}")
        max_tokens = min(params.max_tokens, self.ecfg.max_model_len - len(prompt_ids))
        hold = bool(kv_transfer_params and kv_transfer_params.get("do_remote_decode"))
        if hold:
            max_tokens = 1  # P/D prefill: first token only, KV kept for the decode engine
        iid = next(self._ids)
        req_id = req_id or f"req-{iid}"
        seed = params.seed if params.seed is not None else (iid * 7919 + self.ecfg.seed)
        st = RequestState(req_id, iid, prompt if isinstance(prompt, str) else None, prompt_ids,
                          params, time.time())
        # penalties / log-probs need every token on the host: per-token events
        st.stream = stream or bool(params.stop) or params.has_penalties or \
            params.logprobs is not None
        st.hold_kv = hold
        st.traceparent = traceparent
        with self._lock:
            self.sched.add_request(iid, prompt_ids, max_tokens, params.min_tokens,
                                   params.ignore_eos, list(params.stop_token_ids),
                                   float(params.temperature), float(params.top_p),
                                   int(params.top_k), int(seed), st.stream)
            if hold:
                self.sched.set_hold_kv(iid, True)
            self.reqs[iid] = st
            self.by_name[req_id] = iid
            if params.has_penalties or params.logprobs is not None:
                self._n_extra += 1
        self.metrics.req_total.inc(model_name=self.model_name)
        return req_id

    def abort_request(self, req_id: str) -> bool:
        """Thread-safe abort.  Applied at the next step boundary (never between a step's
        schedule and update), so it can be called from HTTP handler threads."""
        with self._lock:
            iid = self.by_name.get(req_id)
            if iid is None:
                return False
            self._pending_aborts.append(iid)
        return True

    # ------------------------------------------------------------------ P/D
    def held_blocks(self, transfer_id: int) -> list:
        with self._lock:
            return list(self.sched.held_blocks(int(transfer_id)))

    def free_held(self, transfer_id: int) -> None:
        with self._lock:
            self.sched.free_held(int(transfer_id))

    def take_held(self, transfer_id: int) -> list:
        """A send of this transfer's KV starts: its blocks leave the TTL / release path and
        stay owned until finish_transfer() (the send's completion), so neither the TTL sweep
        nor a decode side's /kv/release can recycle blocks that are still being packed."""
        with self._lock:
            return list(self.sched.take_held(int(transfer_id)))

    def finish_transfer(self, transfer_id: int) -> None:
        with self._lock:
            self.sched.finish_transfer(int(transfer_id))

    def reserve_prefilled(self, req_id: str, prompt_ids: list, first_token: int,
                          params: SamplingParams, stream: bool = False):
        """Decode side of P/D: allocate blocks for a remotely prefilled prompt.
        Returns (iid, block_ids); block_ids is empty when the KV pool is short."""
        params = params.normalized()
        prompt_ids = [int(t) for t in prompt_ids]
        max_tokens = min(params.max_tokens, self.ecfg.max_model_len - len(prompt_ids))
        iid = next(self._ids)
        seed = params.seed if params.seed is not None else (iid * 7919 + self.ecfg.seed)
        st = RequestState(req_id, iid, None, prompt_ids, params, time.time())
        # as in add_request: penalties / log-probs need every token on the host
        extra = params.has_penalties or params.logprobs is not None
        st.stream = stream or bool(params.stop) or extra
        st.first_token_time = st.arrival
        st.output_ids = [int(first_token)]
        st.text = self.tokenizer.decode_token(int(first_token)) if st.stream else ""
        with self._lock:
            blocks = self.sched.reserve_prefilled(
                iid, prompt_ids + [int(first_token)], len(prompt_ids), max_tokens,
                params.min_tokens, params.ignore_eos, list(params.stop_token_ids),
                float(params.temperature), float(params.top_p), int(params.top_k), int(seed),
                st.stream)
            if blocks:
                self.reqs[iid] = st
                self.by_name[req_id] = iid
                if extra:  # paired with the decrement on finish / abort
                    self._n_extra += 1
        if blocks:
            self.metrics.req_total.inc(model_name=self.model_name)
        return iid, list(blocks)

    def set_first_token(self, iid: int, tok: int) -> None:
        """P/D streamed hand-off: the first token of a request reserved before it existed."""
        with self._lock:
            self.sched.set_first_token(int(iid), int(tok))
            st = self.reqs.get(int(iid))
            if st is not None:
                st.output_ids = [int(tok)]
                st.text = self.tokenizer.decode_token(int(tok)) if st.stream else ""

    def hold_kv_progress(self) -> list:
        """P/D prefill side: (transfer id, block table, computed tokens) of every request
        whose KV is being prefilled for a remote decode (for streaming finished blocks)."""
        out = []
        with self._lock:
            for iid, st in self.reqs.items():
                if st.hold_kv and not st.finished:
                    info = self.sched.request_info(iid)
                    if info is not None and info["status"] == 1:  # RUNNING
                        out.append((iid, list(self.sched.block_table(iid)),
                                    int(info["num_computed"])))
        return out

    def tail_slot(self, iid: int) -> int:
        """The V-tail slot of a reserved request (assigned now if it has none; -1 = none)."""
        with self._lock:
            return int(self.sched.tail_slot(int(iid)))

    def activate(self, iid: int, tail_filled: bool = False) -> None:
        """tail_filled: the KV hand-off already wrote the request's V tail (the IPC pull
        fills it in the same launch)."""
        with self._lock:
            self.sched.activate(int(iid))
            if self.runner.v_tails is not None and not tail_filled:
                # the prompt's KV arrived whole: its partial last V group -> the V tail
                info = self.sched.request_info(int(iid))
                if info is not None:
                    self.runner.fill_tail(self.sched.tail_slot(int(iid)),
                                          self.sched.block_table(int(iid)),
                                          int(info["num_computed"]))

    def _apply_aborts(self) -> None:
        with self._lock:
            pend, self._pending_aborts = self._pending_aborts, []
            for iid in pend:
                self.sched.abort_request(iid)
                st = self.reqs.pop(iid, None)
                if st is not None:
                    self.by_name.pop(st.req_id, None)
                    st.finished, st.finish_reason = True, "abort"
                    self.metrics.success.inc(model_name=self.model_name, finished_reason="abort")
                    if st.params.has_penalties or st.params.logprobs is not None:
                        self._n_extra -= 1
                self.sched.release(iid)

    def has_unfinished(self) -> bool:
        if self._pending_aborts:
            self._apply_aborts()
        return self.sched.has_work()

    @property
    def num_unfinished(self) -> int:
        return self.sched.num_running + self.sched.num_waiting

    # ------------------------------------------------------------------ step
    def _try_lookahead(self):
        """Launch the next decode step while the current one runs (see
        Scheduler.schedule_lookahead); None when the next step must be a normal one."""
        if not self._async_decode or self._n_extra or self._pending_aborts:
            return None
        with self._lock:
            info = self.sched.schedule_lookahead(self.runner.host_buffers())
        if not info["num_seqs"]:
            return None
        self.lookahead_steps += 1
        return info, self.runner.launch_decode(info, chained=True)

    def step(self) -> list[RequestOutput]:
        t0 = time.time()
        if self._pending_aborts:
            self._apply_aborts()
        sample_pos: dict = {}
        if self._inflight is not None:
            # a lookahead step is already queued: queue the one after it, then collect it
            info, handle = self._inflight
            t1 = time.time()
            self._inflight = self._try_lookahead()
            toks = self.runner.wait_decode(handle)
            self.last_step_mixed = False
        else:
            with self._lock:
                info = self.sched.schedule(self.runner.host_buffers())
            if info["num_preempted"]:
                self.metrics.preempt.inc(info["num_preempted"], model_name=self.model_name)
            self.last_step_mixed = bool(info["is_prefill"] and info.get("num_decode", 0))
            if info["is_prefill"]:  # requests are admitted only in steps with prefill rows
                self._observe_queue_time(info, t0)
            t1 = time.time()
            if info["num_seqs"] == 0:
                # nothing runnable; still flush requests the scheduler had to end (token -1)
                if not self.sched.has_work():
                    return []
                toks = np.zeros(0, dtype=np.int64)
            else:
                if self._n_extra:
                    info["extras"], sample_pos = self._step_extras(info)
                if (self._async_decode and not info["is_prefill"] and "extras" not in info
                        and (not self.runner.buckets
                             or info["num_seqs"] <= self.runner.buckets[-1])):
                    handle = self.runner.launch_decode(info)
                    self._inflight = self._try_lookahead()
                    toks = self.runner.wait_decode(handle)
                else:
                    toks = self.runner.execute(info)
        now = time.time()
        self.timers["schedule"] += t1 - t0
        self.timers["execute"] += now - t1
        if info["num_seqs"]:
            kind = ("mixed" if self.last_step_mixed else "prefill") if info["is_prefill"] \
                else "decode"
            self.step_kinds[kind][0] += now - t1
            self.step_kinds[kind][1] += 1
        with self._lock:
            ids, new, fin, first = self.sched.update(np.ascontiguousarray(toks, dtype=np.int64))
        m, name = self.metrics, self.model_name
        if info["is_prefill"]:
            m.prompt_tokens.inc(info["num_tokens"] - info.get("num_decode", 0), model_name=name)
        # tokens actually appended: rows of requests that ended while the step was in flight
        # (lookahead) are computed but discarded
        m.gen_tokens.inc(self.sched.last_appended, model_name=name)
        m.step_time.observe(now - t0, model_name=name,
                            phase="prefill" if info["is_prefill"] else "decode")
        outs = []
        for iid, tok, f, fst in zip(ids, new, fin, first):
            st = self.reqs.get(iid)
            if st is None:
                continue
            if fst:
                st.first_token_time = now
                m.ttft.observe(now - st.arrival, model_name=name)
            reason = FINISH_REASONS.get(f)
            if tok >= 0 and st.params.logprobs is not None and iid in sample_pos:
                lps = self.runner.last_logprobs
                st.logprobs.append(float(lps[sample_pos[iid]]) if lps is not None else 0.0)
                top = self.runner.last_top
                if st.params.logprobs > 0 and top is not None:
                    k_ = sample_pos[iid]
                    st.top_logprobs.append([(int(t), float(v)) for t, v in
                                            zip(top[0][k_][:st.params.logprobs],
                                                top[1][k_][:st.params.logprobs])])
            if tok < 0:  # ended by the scheduler (KV pool can never hold it): no new token
                delta = ""
            elif st.stream:
                st.output_ids.append(tok)
                delta = "" if (reason == "stop" and tok == self.mcfg.eos_id) else \
                    self.tokenizer.decode_token(tok)
                st.text += delta
                if reason is None and st.params.stop:
                    for s_ in st.params.stop:
                        if s_ and s_ in st.text:
                            cut = st.text.index(s_)
                            delta = delta[: max(0, len(delta) - (len(st.text) - cut))]
                            st.text = st.text[:cut]
                            reason = "stop"
                            with self._lock:
                                self.sched.abort_request(iid)
                            break
            else:
                delta = ""
            cached = 0
            if reason is not None:
                if not st.stream:
                    out_ids = self.sched.output_tokens(iid)
                    if reason == "stop" and out_ids and out_ids[-1] == self.mcfg.eos_id:
                        st.text = self.tokenizer.decode(out_ids[:-1])
                    else:
                        st.text = self.tokenizer.decode(out_ids)
                    st.output_ids = list(out_ids)
                    delta = st.text
                st.finished, st.finish_reason = True, reason
                n = len(st.output_ids)
                m.success.inc(model_name=name, finished_reason=reason)
                m.e2e.observe(now - st.arrival, model_name=name)
                m.duration.observe(now - st.arrival, model_name=name)
                if n > 1 and st.first_token_time is not None:
                    m.tpot.observe((now - st.first_token_time) / (n - 1), model_name=name)
                info_r = self.sched.request_info(iid)
                cached = info_r["num_cached"] if info_r else 0
                tr = tracing.get_tracer()
                if tr is not None:
                    tracing.record_request(
                        tr, req_id=st.req_id, model=name, arrival=st.arrival,
                        first_token=st.first_token_time, finish=now,
                        prompt_tokens=len(st.prompt_ids), completion_tokens=n,
                        finish_reason=reason, max_tokens=st.params.max_tokens,
                        temperature=st.params.temperature, top_p=st.params.top_p,
                        traceparent=st.traceparent, cached_tokens=cached)
                with self._lock:
                    self.sched.release(iid)
                    self.reqs.pop(iid, None)
                    self.by_name.pop(st.req_id, None)
                    if st.params.has_penalties or st.params.logprobs is not None:
                        self._n_extra -= 1
            elif not st.stream:
                continue  # first-token event of a non-streaming request: metrics only
            kvp = None
            if st.hold_kv and st.finished and st.output_ids:  # (an aborted prompt hands off nothing)
                kvp = {"transfer_id": iid, "num_prompt": len(st.prompt_ids),
                       "prompt_token_ids": st.prompt_list(), "first_token": st.output_ids[0],
                       "remote_rank": self.rank, "num_blocks": len(self.sched.held_blocks(iid)),
                       "group": self.pd_group}
            outs.append(RequestOutput(st.req_id, st.prompt_list(), st.output_ids, [tok], st.text,
                                      delta, st.finished, st.finish_reason,
                                      (st.first_token_time - st.arrival)
                                      if st.first_token_time else None, cached, kvp,
                                      list(st.logprobs) if st.params.logprobs is not None
                                      else None,
                                      list(st.top_logprobs) if st.params.logprobs else None))
        self.steps += 1
        self._update_gauges()
        self.timers["post"] += time.time() - now
        return outs

    def _observe_queue_time(self, info: dict, t_sched: float) -> None:
        """vllm:request_queue_time_seconds: arrival -> first scheduled (prefill rows only)."""
        ids = self.runner.np["req_ids"]
        for s_ in range(info.get("num_decode", 0), info["num_seqs"]):
            st = self.reqs.get(int(ids[s_]))
            if st is not None and st.first_scheduled is None:
                st.first_scheduled = t_sched
                self.metrics.queue.observe(max(0.0, t_sched - st.arrival),
                                           model_name=self.model_name)

    def _step_extras(self, info: dict):
        """Penalty COO + log-prob flag for the sampled rows of this step (host side; only
        called while some live request uses penalties or log-probs)."""
        npb = self.runner.np
        rows, toks, counts = [], [], []
        B = info["num_seqs"]
        ns = info["num_samples"]
        pres = np.zeros(max(ns, 1), np.float32)
        freq = np.zeros(max(ns, 1), np.float32)
        rep = np.ones(max(ns, 1), np.float32)
        want_lp, ntop = False, 0
        pos: dict = {}
        k = 0
        for s_ in range(B):
            if not npb["sample_mask"][s_]:
                continue
            iid = int(npb["req_ids"][s_])
            pos[iid] = k
            st = self.reqs.get(iid)
            if st is not None:
                p = st.params
                want_lp |= p.logprobs is not None
                ntop = max(ntop, p.logprobs or 0)
                if p.has_penalties:
                    pres[k], freq[k], rep[k] = (p.presence_penalty, p.frequency_penalty,
                                                p.repetition_penalty)
                    cnt: dict = {}
                    for t in st.output_ids:
                        cnt[t] = cnt.get(t, 0) + 1
                    if p.repetition_penalty != 1.0:
                        for t in st.prompt_list():
                            cnt.setdefault(t, 0)
                    for t, c in cnt.items():
                        rows.append(k)
                        toks.append(t)
                        counts.append(c)
            k += 1
        extras = {"logprobs": want_lp, "top_logprobs": ntop}
        if rows:
            extras["penalties"] = (np.asarray(rows, np.int32), np.asarray(toks, np.int32),
                                   np.asarray(counts, np.int32), pres, freq, rep)
        return extras, pos

    def _update_gauges(self) -> None:
        m, name = self.metrics, self.model_name
        m.running.set(self.sched.num_running, model_name=name)
        m.waiting.set(self.sched.num_waiting, model_name=name)
        m.active.set(self.sched.num_running + self.sched.num_waiting, model_name=name)
        m.kv_usage.set(self.sched.kv_usage(), model_name=name)
        hits, queries = self.sched.prefix_stats()
        m.prefix_hits.set_total(hits, model_name=name)
        m.prefix_queries.set_total(queries, model_name=name)
        m.kv_held.set(self.sched.num_held, model_name=name)
        m.kv_held_expired.set_total(self.sched.held_expired_total, model_name=name)
        agent = self.kv_agent
        if agent is not None:
            m.kv_xfer_fail.set_total(agent.failures, model_name=name)
            m.kv_broken.set(1.0 if agent.broken else 0.0, model_name=name)
            m.kv_resets.set_total(agent.resets, model_name=name)
            m.kv_xfer_bytes.set_total(agent.bytes_sent, model_name=name, direction="send")
            m.kv_xfer_bytes.set_total(agent.bytes_recv, model_name=name, direction="recv")
            from ..parallel.kv_transfer import CHANNEL_PROBES

            for peer, pr in list(CHANNEL_PROBES.items()):
                m.kv_probe_gbps.set(round(pr["gbps"], 3), model_name=name, peer=peer,
                                    transport=pr["transport"], role=pr["role"])
            probe = getattr(self, "kv_ipc_state", None)  # set by the serving layer (decode)
            m.kv_ipc.set(1.0 if probe is not None and probe() else 0.0, model_name=name)

    # ------------------------------------------------------------------ offline API
    def generate(self, prompts: Iterable, params: Optional[SamplingParams] = None,
                 prompt_ids: Optional[list] = None) -> list[RequestOutput]:
        names = []
        params = (params or SamplingParams()).normalized()  # once for the whole batch
        if prompt_ids is not None:
            for p in prompt_ids:
                names.append(self._add(None, None, params, p))
        else:
            for p in prompts:
                names.append(self._add(None, p, params, None))
        final: dict[str, RequestOutput] = {}
        while self.has_unfinished():
            for o in self.step():
                if o.finished:
                    final[o.req_id] = o
        return [final[n] for n in names if n in final]
