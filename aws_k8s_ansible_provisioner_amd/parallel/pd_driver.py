"""In-process disaggregated prefill/decode pair (no HTTP): the P/D data path of the
`pd` deployment preset driven directly, for `bench.py --mode pd` and tests.

Ranks [0, W/2) are prefill engines, ranks [W/2, W) decode engines; prefill rank i feeds
decode rank i + W/2.  After every prefill STEP:
  prefill rank: ONE metadata message on a gloo control group naming every hand-off entry
                of the step, then ONE `KVTransferAgent.send_packed` of all their blocks
                (packed by `kv_gather` on the compute stream, sent by the agent thread over
                RCCL while the next prefill step runs).  Entries:
                  CHUNK  (streamed mode, the default) blocks of a still-prefilling prompt
                         that became complete in this step -- a long prompt's KV moves
                         chunk by chunk WHILE its later chunks are computed;
                  FINAL  the request finished its prefill (first token sampled): its
                         remaining blocks + the first token.
                With streaming off (`chunked=False`) only FINAL entries exist and each
                carries every block of the prompt (whole-prompt hand-off).
  decode rank:  metadata -> `reserve_prefilled` on a request's first entry -> ONE
                `recv_blocks` of the step's blocks into the reserved ids -> on FINAL:
                `set_first_token` + `activate` -> continuous-batching decode.
Metadata and KV go in the same order on both sides, so the sends and recvs pair up.

TTFT is taken on the decode side (when the request becomes decodable with its first
token), i.e. it includes prefill, queueing and the KV hand-off.
"""
from __future__ import annotations

import threading
import time
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from ..engine.config import SamplingParams
from .kv_transfer import KVTransferAgent

_END = -1
_CHUNK, _FINAL = 0, 1


def _send_msg(arr: np.ndarray, dst: int, group) -> None:
    t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int64))
    dist.send(torch.tensor([t.numel()], dtype=torch.int64), dst, group=group)
    if t.numel():
        dist.send(t, dst, group=group)


def _recv_msg(src: int, group) -> np.ndarray:
    n = torch.empty(1, dtype=torch.int64)
    dist.recv(n, src, group=group)
    t = torch.empty(int(n.item()), dtype=torch.int64)
    if t.numel():
        dist.recv(t, src, group=group)
    return t.numpy()


class PDPair:
    def __init__(self, engine, rank: int, world: int, ctrl_group=None, data_group=None):
        if world < 2 or world % 2:
            raise ValueError("P/D needs an even number of ranks (prefill half + decode half)")
        self.engine = engine
        self.rank, self.world = rank, world
        self.is_prefill = rank < world // 2
        self.peer = rank + world // 2 if self.is_prefill else rank - world // 2
        self.ctrl = ctrl_group
        self.agent = KVTransferAgent(engine.runner.kv, group=data_group)
        self.batches = 0

    # ------------------------------------------------------------------ prefill side
    def run_prefill(self, prompts: list[list[int]], params: SamplingParams,
                    chunked: bool = True) -> dict:
        eng = self.engine
        names = [eng.add_request(None, None, params, prompt_ids=p,
                                 kv_transfer_params={"do_remote_decode": True})
                 for p in prompts]
        prompt_of = {}
        pending = []
        sent = 0
        streamed: dict = {}  # transfer id -> blocks already sent
        bs = eng.ecfg.block_size
        while eng.has_unfinished():
            outs = eng.step()
            entries, blocks, tids_done = [], [], []
            if chunked:
                for iid, bt, computed in eng.hold_kv_progress():
                    full = min(computed // bs, len(bt))
                    s0 = streamed.get(iid, 0)
                    if full > s0:
                        new = iid not in prompt_of
                        if new:
                            prompt_of[iid] = eng.reqs[iid].prompt_ids
                        entries.append((_CHUNK, iid, prompt_of[iid] if new else None, -1, s0,
                                        full - s0))
                        blocks += bt[s0:full]
                        streamed[iid] = full
            for o in outs:
                if not (o.finished and o.kv_transfer_params):
                    continue
                tid = int(o.kv_transfer_params["transfer_id"])
                b = eng.take_held(tid)
                s0 = streamed.pop(tid, 0)
                new = tid not in prompt_of
                entries.append((_FINAL, tid, list(o.prompt_ids) if new else None,
                                int(o.output_ids[0]), s0, len(b) - s0))
                prompt_of.pop(tid, None)
                blocks += b[s0:]
                tids_done.append(tid)
                sent += 1
            if not entries:
                continue
            msg = [len(entries)]
            for kind, tid, prompt, first, b0, nb in entries:
                msg += [kind, tid, -1 if prompt is None else len(prompt), first, b0, nb]
                if prompt is not None:
                    msg += list(prompt)
            _send_msg(np.array(msg, dtype=np.int64), self.peer, self.ctrl)
            # packed on the compute stream now: the finished requests' blocks can be freed
            # at once (any reuse is a later kernel of the same stream)
            packed = self.agent.gather(blocks) if blocks else None
            for t in tids_done:
                eng.finish_transfer(t)
            if packed is not None:
                pending.append(self.agent.send_packed(packed, self.peer))
        _send_msg(np.array([_END], dtype=np.int64), self.peer, self.ctrl)
        for ev in pending:
            ev.wait()
            if ev.box.get("err") is not None:
                raise ev.box["err"]
        return {"requests": len(names), "sent": sent, "transfers": len(pending)}

    # ------------------------------------------------------------------ decode side
    def run_decode(self, params: SamplingParams, t0: Optional[float] = None) -> dict:
        eng = self.engine
        t0 = t0 if t0 is not None else time.time()
        ttft: list[float] = []
        done = threading.Event()
        errors: list[BaseException] = []

        def receiver():
            try:
                k = 0
                mine: dict = {}  # prefill transfer id -> (decode iid, reserved blocks)
                while True:
                    msg = _recv_msg(self.peer, self.ctrl)
                    if msg[0] == _END:
                        return
                    off, dst, finals = 1, [], []
                    for _ in range(int(msg[0])):
                        kind, tid, n_prompt, first, b0, nb = (int(x) for x in msg[off:off + 6])
                        off += 6
                        if n_prompt >= 0:
                            prompt = [int(x) for x in msg[off:off + n_prompt]]
                            off += n_prompt
                            if tid not in mine:
                                iid, blocks = eng.reserve_prefilled(
                                    f"pd-{self.rank}-{k}", prompt, max(first, 0), params)
                                if not blocks:
                                    raise RuntimeError("decode KV pool short")
                                mine[tid] = (iid, blocks)
                                k += 1
                        iid, blocks = mine[tid]
                        if b0 + nb > len(blocks):
                            raise RuntimeError(f"hand-off of blocks [{b0}, {b0 + nb}) past the "
                                               f"{len(blocks)} reserved")
                        dst += blocks[b0:b0 + nb]
                        if kind == _FINAL:
                            finals.append((tid, iid, first))
                    if dst:
                        self.agent.recv_blocks(dst, self.peer)
                    for tid, iid, first in finals:
                        eng.set_first_token(iid, first)
                        eng.activate(iid)
                        ttft.append(time.time() - t0)
                        mine.pop(tid)
                    self.batches += 1
            except BaseException as e:  # surfaced to the caller
                errors.append(e)
            finally:
                done.set()

        th = threading.Thread(target=receiver, name="pd-recv", daemon=True)
        th.start()
        out_tokens = 0
        n_done = 0
        while not (done.is_set() and not eng.has_unfinished()):
            if errors:
                break
            if not eng.has_unfinished():
                time.sleep(0.0005)
                continue
            for o in eng.step():
                if o.finished:
                    out_tokens += len(o.output_ids)
                    n_done += 1
        th.join()
        if errors:
            raise errors[0]
        return {"output_tokens": out_tokens, "finished": n_done, "ttft": ttft}

    def close(self) -> None:
        self.agent.close()
