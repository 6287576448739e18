"""In-process disaggregated prefill/decode pair (no HTTP): the P/D data path of the
`pd` deployment preset driven directly, for `bench.py --mode pd` and tests.

Ranks [0, W/2) are prefill engines, ranks [W/2, W) decode engines; prefill rank i feeds
decode rank i + W/2.  Per request:
  prefill rank: prefill + first token (KV held in its pool, `hold_kv`) -> metadata message
                on a gloo control group -> `KVTransferAgent.send_blocks` (kv_gather + one
                RCCL send over xGMI) -> its blocks are freed when the send completes;
  decode rank:  metadata -> `reserve_prefilled` (blocks + first token) -> `recv_blocks`
                (one RCCL recv + kv_scatter) -> `activate` -> continuous-batching decode.
Metadata and KV go in the same order on both sides, so the RCCL sends and recvs pair up.

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

    # ------------------------------------------------------------------ prefill side
    def run_prefill(self, prompts: list[list[int]], params: SamplingParams) -> dict:
        eng = self.engine
        names = [eng.add_request(None, None, params, prompt_ids=p,
                                 kv_transfer_params={"do_remote_decode": True})
                 for p in prompts]
        pending = []
        sent = 0
        while eng.has_unfinished():
            for o in eng.step():
                if not o.finished or not o.kv_transfer_params:
                    continue
                kvp = o.kv_transfer_params
                tid = int(kvp["transfer_id"])
                blocks = eng.held_blocks(tid)
                msg = np.array([tid, len(o.prompt_ids), int(o.output_ids[0]), len(blocks)]
                               + list(o.prompt_ids), dtype=np.int64)
                _send_msg(msg, self.peer, self.ctrl)
                pending.append(self.agent.send_blocks(
                    blocks, self.peer, on_done=lambda t=tid: eng.free_held(t), wait=False))
                sent += 1
        _send_msg(np.array([_END], dtype=np.int64), self.peer, self.ctrl)
        for ev in pending:
            ev.wait()
        return {"requests": len(names), "sent": sent}

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
                while True:
                    msg = _recv_msg(self.peer, self.ctrl)
                    if msg[0] == _END:
                        return
                    tid, n_prompt, first, nblk = (int(x) for x in msg[:4])
                    prompt = [int(x) for x in msg[4:4 + n_prompt]]
                    iid, blocks = eng.reserve_prefilled(f"pd-{self.rank}-{k}", prompt, first,
                                                        params)
                    if len(blocks) != nblk:
                        raise RuntimeError(f"decode pool short: {len(blocks)} vs {nblk} blocks")
                    self.agent.recv_blocks(blocks, self.peer)
                    eng.activate(iid)
                    ttft.append(time.time() - t0)
                    k += 1
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
