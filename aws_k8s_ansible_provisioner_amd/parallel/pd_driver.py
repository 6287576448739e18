"""In-process disaggregated prefill/decode pair (no HTTP): the P/D data path of the
`pd` deployment preset driven directly, for `bench.py --mode pd` and tests.

Ranks [0, W/2) are prefill engines, ranks [W/2, W) decode engines; prefill rank i feeds
decode rank i + W/2.  Per prefill STEP (every request whose prefill finished in it):
  prefill rank: prefill + first token (KV held in its pool, `hold_kv`) -> ONE metadata
                message for the step's requests on a gloo control group -> ONE
                `KVTransferAgent.send_blocks` of all their blocks (kv_gather + one RCCL send
                over xGMI) -> the blocks are freed when the send ends;
  decode rank:  metadata -> `reserve_prefilled` per request -> ONE `recv_blocks` of the
                concatenated block lists (one RCCL recv + kv_scatter) -> `activate` each ->
                continuous-batching decode.
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
        self.batches = 0

    # ------------------------------------------------------------------ prefill side
    def run_prefill(self, prompts: list[list[int]], params: SamplingParams) -> dict:
        eng = self.engine
        names = [eng.add_request(None, None, params, prompt_ids=p,
                                 kv_transfer_params={"do_remote_decode": True})
                 for p in prompts]
        pending = []
        sent = 0
        while eng.has_unfinished():
            batch = [o for o in eng.step() if o.finished and o.kv_transfer_params]
            if not batch:
                continue
            msg, tids, blocks = [len(batch)], [], []
            for o in batch:
                tid = int(o.kv_transfer_params["transfer_id"])
                b = eng.take_held(tid)
                msg += [tid, len(o.prompt_ids), int(o.output_ids[0]), len(b)] + list(o.prompt_ids)
                tids.append(tid)
                blocks += b
            _send_msg(np.array(msg, dtype=np.int64), self.peer, self.ctrl)
            pending.append(self.agent.send_blocks(
                blocks, self.peer, on_done=lambda ts=tuple(tids): [eng.finish_transfer(t) for t in ts],
                wait=False))
            sent += len(batch)
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
                while True:
                    msg = _recv_msg(self.peer, self.ctrl)
                    if msg[0] == _END:
                        return
                    off, reserved = 1, []
                    for _ in range(int(msg[0])):
                        tid, n_prompt, first, nblk = (int(x) for x in msg[off:off + 4])
                        prompt = [int(x) for x in msg[off + 4:off + 4 + n_prompt]]
                        off += 4 + n_prompt
                        iid, blocks = eng.reserve_prefilled(f"pd-{self.rank}-{k}", prompt,
                                                            first, params)
                        if len(blocks) != nblk:
                            raise RuntimeError(f"decode pool short: {len(blocks)} vs {nblk} "
                                               "blocks")
                        reserved.append((iid, blocks))
                        k += 1
                    self.agent.recv_blocks([b for _, bl in reserved for b in bl], self.peer)
                    for iid, _ in reserved:
                        eng.activate(iid)
                        ttft.append(time.time() - t0)
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
