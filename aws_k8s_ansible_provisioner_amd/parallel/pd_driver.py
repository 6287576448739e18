"""In-process disaggregated prefill/decode group (no HTTP): the P/D data path of the `pd`
deployment preset driven directly, for `bench.py --mode pd` and tests.

Layout (N prefill : M decode ranks, M a multiple of N): ranks [0, N) are prefill engines,
ranks [N, N+M) decode engines; decode rank N + j takes its requests from prefill rank j % N,
so prefill rank i feeds the M/N decode ranks N + i, N + i + N, ...  It hands each request to
one of them (round robin, chosen when the request's first KV goes out).  The default is
N = M = W/2 (1:1 pairs).

After every prefill STEP the prefill rank sends, per destination decode rank, ONE metadata
message on a gloo control group naming every hand-off entry of the step:
  CHUNK  (streamed mode, the default) blocks of a still-prefilling prompt that became
         complete in this step -- a long prompt's KV moves chunk by chunk WHILE its later
         chunks are computed;
  FINAL  the request finished its prefill (first token sampled): its remaining blocks + the
         first token.
With streaming off (`chunked=False`) only FINAL entries exist and each carries every block
of the prompt (whole-prompt hand-off).

Two transports for the KV itself (`transport`):
  "ipc"  (GPU default) the decode rank mapped the prefill rank's whole KV cache once through
         hipIpc (KVTransferAgent.connect_ipc); a message carries the prefill-side block ids
         and the decode rank moves the blocks with ONE kv_pull launch per message (peer cache
         -> its own reserved blocks, V tails of the finished requests filled in the same
         launch), then acknowledges the FINAL entries on an ack group; the prefill rank
         keeps those requests' blocks leased until the ack (finish_transfer).
  "p2p"  (CPU / gloo, or AKAP_KV_TRANSPORT=p2p) ONE `KVTransferAgent.send_packed` of all the
         message's blocks (packed by `kv_gather` on the compute stream, sent by the agent
         thread while the next prefill step runs) matched by one `recv_blocks` that unpacks
         into the reserved ids; the blocks are freed as soon as they are packed.
Metadata and KV go in the same order on both sides of each pair, so sends and recvs pair up.

TTFT is taken on the decode side (when the request becomes decodable with its first
token), i.e. it includes prefill, queueing and the KV hand-off.
"""
from __future__ import annotations

import os
import threading
import time
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from ..engine.config import SamplingParams
from .kv_transfer import KVIpcOpenTimeout, KVTransferAgent

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


def pd_layout(world: int, prefill_ranks: Optional[int] = None) -> tuple[int, int]:
    """(N prefill, M decode) ranks of a P/D job of `world` ranks; M % N == 0."""
    n = world // 2 if not prefill_ranks else int(prefill_ranks)
    m = world - n
    if n < 1 or m < 1 or m % n:
        raise ValueError(f"P/D layout {n} prefill : {m} decode ranks: needs N >= 1, M >= 1 "
                         f"and M a multiple of N")
    return n, m


def default_transport(engine) -> str:
    env = os.environ.get("AKAP_KV_TRANSPORT", "auto")
    if env in ("ipc", "p2p"):
        return env
    return "ipc" if engine.runner.is_gpu else "p2p"


class PDPair:
    def __init__(self, engine, rank: int, world: int, ctrl_group=None, data_group=None,
                 prefill_ranks: Optional[int] = None, transport: Optional[str] = None,
                 ack_group=None):
        """Collective over the job: every rank constructs its PDPair (the ack group and the
        IPC handle exchange are made here)."""
        if world < 2:
            raise ValueError("P/D needs at least 2 ranks (prefill + decode)")
        self.n_prefill, self.n_decode = pd_layout(world, prefill_ranks)
        self.engine = engine
        self.rank, self.world = rank, world
        self.is_prefill = rank < self.n_prefill
        N = self.n_prefill
        if self.is_prefill:
            self.peers = list(range(N + rank, world, N))
            self.peer = self.peers[0]
        else:
            self.peer = (rank - N) % N
            self.peers = [self.peer]
        self.ctrl = ctrl_group
        self.transport = transport or default_transport(engine)
        self.agent = KVTransferAgent(engine.runner.kv_segs, group=data_group)
        self.batches = 0
        self.pull_seconds = 0.0
        self.pulled_bytes = 0
        self.ack = None
        if self.transport == "ipc":
            # acknowledgements of pulled FINAL entries flow decode -> prefill on their own
            # group (the ctrl group's messages flow the other way, from another thread)
            self.ack = ack_group if ack_group is not None else dist.new_group(backend="gloo")
            if self.is_prefill:
                meta = [self.agent.ipc_meta()]
                for p in self.peers:
                    dist.send_object_list(meta, p, group=self.ctrl)
            else:
                meta = [None]
                dist.recv_object_list(meta, self.peer, group=self.ctrl)
            # a mapping that does not return in time (bounded: KVTransferAgent.connect_ipc)
            # moves the WHOLE job to the p2p transport -- every rank must agree before the
            # first hand-off, since the two transports pair differently
            ok = 1
            if not self.is_prefill:
                try:
                    self.agent.connect_ipc(meta[0])
                except KVIpcOpenTimeout:
                    ok = 0
            flag = torch.tensor([ok], dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.ctrl)
            if not int(flag.item()):
                if rank == 0:
                    print("[pd] hipIpc mapping timed out on a decode rank: the job uses the "
                          "p2p transport", flush=True)
                self.transport = "p2p"

    # ------------------------------------------------------------------ prefill side
    def run_prefill(self, prompts: list[list[int]], params: SamplingParams,
                    chunked: bool = True) -> dict:
        eng = self.engine
        ipc = self.transport == "ipc"
        names = [eng.add_request(None, None, params, prompt_ids=p,
                                 kv_transfer_params={"do_remote_decode": True})
                 for p in prompts]
        prompt_of = {}
        pending = []
        sent = 0
        streamed: dict = {}  # transfer id -> blocks already handed off
        dest: dict = {}      # transfer id -> decode rank
        rr = [0]
        bs = eng.ecfg.block_size
        ack_errs: list = []
        ack_threads = []

        def dest_of(tid):
            if tid not in dest:
                dest[tid] = self.peers[rr[0] % len(self.peers)]
                rr[0] += 1
            return dest[tid]

        def ack_loop(peer):
            """Lease releases: every FINAL the decode rank pulled frees its blocks here."""
            try:
                while True:
                    msg = _recv_msg(peer, self.ack)
                    if msg.size == 1 and msg[0] == _END:
                        return
                    for t in msg:
                        eng.finish_transfer(int(t))
            except BaseException as e:
                ack_errs.append(e)

        if ipc:
            for p in self.peers:
                th = threading.Thread(target=ack_loop, args=(p,), name=f"pd-ack-{p}",
                                      daemon=True)
                th.start()
                ack_threads.append(th)
        while eng.has_unfinished():
            outs = eng.step()
            per: dict = {p: ([], []) for p in self.peers}  # peer -> (entries, blocks)
            tids_done = []
            if chunked:
                for iid, bt, computed in eng.hold_kv_progress():
                    full = min(computed // bs, len(bt))
                    s0 = streamed.get(iid, 0)
                    if full > s0:
                        new = iid not in prompt_of
                        if new:
                            prompt_of[iid] = eng.reqs[iid].prompt_list()
                        ents, blks = per[dest_of(iid)]
                        ents.append((_CHUNK, iid, prompt_of[iid] if new else None, -1, s0,
                                     full - s0, bt[s0:full]))
                        blks += bt[s0:full]
                        streamed[iid] = full
            for o in outs:
                if not (o.finished and o.kv_transfer_params):
                    continue
                tid = int(o.kv_transfer_params["transfer_id"])
                b = eng.take_held(tid)
                s0 = streamed.pop(tid, 0)
                new = tid not in prompt_of
                ents, blks = per[dest_of(tid)]
                ents.append((_FINAL, tid, list(o.prompt_ids) if new else None,
                             int(o.output_ids[0]), s0, len(b) - s0, b[s0:]))
                prompt_of.pop(tid, None)
                blks += b[s0:]
                tids_done.append(tid)
                sent += 1
            for peer, (entries, blocks) in per.items():
                if not entries:
                    continue
                msg = [len(entries)]
                for kind, tid, prompt, first, b0, nb, src in entries:
                    msg += [kind, tid, -1 if prompt is None else len(prompt), first, b0, nb]
                    if prompt is not None:
                        msg += list(prompt)
                    if ipc:
                        msg += [int(x) for x in src]  # the decode rank pulls these blocks
                _send_msg(np.array(msg, dtype=np.int64), peer, self.ctrl)
                if not ipc and blocks:
                    # packed on the compute stream now: the finished requests' blocks can be
                    # freed at once (any reuse is a later kernel of the same stream)
                    pending.append(self.agent.send_packed(self.agent.gather(blocks), peer))
            if not ipc:
                for t in tids_done:
                    eng.finish_transfer(t)
            for t in tids_done:
                dest.pop(t, None)
        for p in self.peers:
            _send_msg(np.array([_END], dtype=np.int64), p, self.ctrl)
        for ev in pending:
            ev.wait()
            if ev.box.get("err") is not None:
                raise ev.box["err"]
        for th in ack_threads:
            th.join()
        if ack_errs:
            raise ack_errs[0]
        return {"requests": len(names), "sent": sent, "transfers": len(pending)}

    # ------------------------------------------------------------------ decode side
    def run_decode(self, params: SamplingParams, t0: Optional[float] = None) -> dict:
        eng = self.engine
        ipc = self.transport == "ipc"
        runner = eng.runner
        model = runner.model
        bs = eng.ecfg.block_size
        t0 = t0 if t0 is not None else time.time()
        ttft: list[float] = []
        done = threading.Event()
        errors: list[BaseException] = []

        def receiver():
            try:
                k = 0
                mine: dict = {}  # prefill transfer id -> (iid, reserved blocks, src blocks, n)
                while True:
                    msg = _recv_msg(self.peer, self.ctrl)
                    if msg[0] == _END:
                        if ipc:
                            _send_msg(np.array([_END], dtype=np.int64), self.peer, self.ack)
                        return
                    off, dst, pairs, finals, tails = 1, [], [], [], []
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
                                mine[tid] = [iid, blocks, [], len(prompt)]
                                k += 1
                        iid, blocks, srcs, n = mine[tid]
                        if b0 + nb > len(blocks):
                            raise RuntimeError(f"hand-off of blocks [{b0}, {b0 + nb}) past the "
                                               f"{len(blocks)} reserved")
                        if ipc:
                            src = [int(x) for x in msg[off:off + nb]]
                            off += nb
                            srcs += src
                            pairs += list(zip(src, blocks[b0:b0 + nb]))
                        else:
                            dst += blocks[b0:b0 + nb]
                        if kind == _FINAL:
                            finals.append((tid, iid, first))
                            if ipc and runner.v_tails is not None and n % 8:
                                # the prompt's partial last V group -> the V tail, same launch
                                slot = eng.tail_slot(iid)
                                g0 = n & ~7
                                if slot >= 0:
                                    tails.append((srcs[g0 // bs], (g0 % bs) // 8, n % 8, slot))
                    if ipc and (pairs or tails):
                        self.pull_seconds += self.agent.pull(
                            pairs, model.hkv, bs, model.D, tail=getattr(runner, "_tail", None),
                            tail_jobs=tails)
                        self.pulled_bytes += self.agent.nbytes(len(pairs))
                    elif dst:
                        self.agent.recv_blocks(dst, self.peer)
                    for tid, iid, first in finals:
                        eng.set_first_token(iid, first)
                        eng.activate(iid, tail_filled=ipc)
                        ttft.append(time.time() - t0)
                        mine.pop(tid)
                    if ipc and finals:
                        _send_msg(np.array([t for t, _, _ in finals], dtype=np.int64),
                                  self.peer, self.ack)
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
