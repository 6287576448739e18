"""KV-cache hand-off between a prefill engine and a decode engine (disaggregated P/D).

MI355X design: the prefill and decode engines are two processes (two GPUs of the same
xGMI mesh) in one torch.distributed group (RCCL).  The KV cache of a BATCH of requests --
all layers, K and V, only their own blocks -- is packed by the `kv_gather` HIP kernel into ONE
contiguous buffer [2L, nblk, block_elems] and moved with a single RCCL send/recv (one large
P2P transfer instead of 2*L*nblk small ones, and one per batch of requests finished in the
same prefill step instead of one per request), then unpacked into the decode engine's own
block ids by `kv_scatter`.  Transfers run on a dedicated stream and thread on each side, so
they overlap both engines' compute.

For Llama-3-8B (32 layers, 8 kv heads x 128, bf16) a 2048-token prompt is 256 MiB of KV:
~2 ms over one xGMI link pair.

Failure handling (a peer that dies or never posts its half must not hang the other):
every send/recv is posted asynchronously (isend/irecv) and waited with a deadline
(`timeout_s`, default AKAP_KV_TIMEOUT_S = 60).  On expiry the transfer raises
KVTransferTimeout and the agent is marked broken: an un-matched P2P op may still be posted in
the communicator, so later transfers on this channel fail fast instead of pairing with stale
ops.  A broken channel is REBUILT, not abandoned: `reset(generation)` -- called on both sides,
coordinated over HTTP (the decode side POSTs /kv/reset to the prefill server and resets its
own agent at the same time) -- creates a fresh process group over the same ranks (a new RCCL
communicator; the stale ops stay behind in the old one) and clears the broken state.
Generations are monotonic, so a repeated or crossed reset request is a no-op.  A send's
`on_done` (the prefill side's finish_transfer) runs whether the send succeeded or not.

Control plane: the decode side asks the prefill server (HTTP POST /kv/push) to send the
blocks of one or more transfer ids to its rank, then posts the matching recv.  The same
code runs on CPU with the gloo backend (tests).

hipIpc PULL transport (the default between GPU engines of one node, AKAP_KV_TRANSPORT=ipc):
the prefill engine exports its whole KV cache ONCE (`ipc_meta`: a hipIpc handle of the
cache allocation + the cache geometry) and the decode engine maps it (`connect_ipc`).  A
hand-off is then one `kv_pull` kernel on the decode GPU that reads the request's blocks
straight out of the peer cache (xGMI, or the same HBM when both engines share a GPU) into
its own block ids and fills the request's V tail in the same launch: no pack, no send /
recv pairing, no unpack, no host staging.  The prefill keeps the blocks leased until the
decode acknowledges the pull (HTTP POST /kv/done, or the PDPair ack channel).
"""
from __future__ import annotations

import datetime
import os
import queue
import threading
import time
from typing import Callable, Optional

import torch
import torch.distributed as dist

from .. import ops

DEFAULT_TIMEOUT_S = float(os.environ.get("AKAP_KV_TIMEOUT_S", "60"))


class KVTransferTimeout(TimeoutError):
    pass


class KVChannelBroken(RuntimeError):
    pass


def _wait(work, timeout_s: float, what: str, gloo: bool) -> None:
    """Bounded wait on an async P2P op.  gloo: its send/recv work completes inside wait(),
    which takes the deadline itself.  RCCL: poll the op's completion event against the
    deadline (wait() would only order the op on the current stream)."""
    if gloo:
        try:
            work.wait(datetime.timedelta(seconds=timeout_s))
        except RuntimeError as e:
            if "imed out" in str(e) or "imeout" in str(e):
                raise KVTransferTimeout(f"{what} did not complete within {timeout_s:.1f}s")
            raise
        return
    deadline = time.monotonic() + timeout_s
    sleep = 0.0001
    while not work.is_completed():
        if time.monotonic() > deadline:
            raise KVTransferTimeout(f"{what} did not complete within {timeout_s:.1f}s")
        time.sleep(sleep)
        sleep = min(sleep * 2, 0.005)
    work.wait()  # surfaces a failed op (raises) and orders the op on the current stream


class KVTransferAgent:
    def __init__(self, kv_cache: torch.Tensor, group=None, timeout_s: float = DEFAULT_TIMEOUT_S):
        """kv_cache: the engine's [L, 2, NB, block_elems] cache tensor (bf16, or uint8 fp8
        bytes -- moved as bf16 pairs: the copy kernels are dtype-agnostic 16-byte moves)."""
        if kv_cache.dtype == torch.uint8:
            kv_cache = kv_cache.view(torch.bfloat16)
        self.kv = kv_cache
        L, two, NB, be = kv_cache.shape
        self.planes = kv_cache.view(L * two, NB, be)
        self.block_elems = be
        self.group = group
        self.timeout_s = timeout_s
        self.device = kv_cache.device
        self.is_gpu = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.device) if self.is_gpu else None
        self._q: "queue.Queue" = queue.Queue()
        self._thread = threading.Thread(target=self._run, name="kv-transfer", daemon=True)
        self._thread.start()
        self.bytes_sent = 0
        self.bytes_recv = 0
        self.transfers = 0
        self.failures = 0
        self.broken: Optional[str] = None
        self.generation = 0  # bumped by every rebuild of the transfer group
        self.resets = 0
        # gloo moves host tensors only: GPU caches on a gloo group (single-GPU rehearsal of
        # the P/D path) stage through pinned host memory
        self.gloo = dist.is_initialized() and dist.get_backend(group) == "gloo"
        self.host_staging = self.is_gpu and self.gloo
        self.peers: dict = {}  # hipIpc: peer key -> (mapped cache address, blocks, plane stride)
        self.pull_seconds = 0.0

    def nbytes(self, nblk: int) -> int:
        return self.planes.shape[0] * nblk * self.block_elems * self.kv.element_size()

    # ---------------------------------------------------------------- worker
    def _run(self) -> None:
        while True:
            job = self._q.get()
            if job is None:
                return
            fn, done = job
            try:
                done(fn(), None)
            except Exception as e:  # surfaced to the waiter
                done(None, e)

    def _submit(self, fn: Callable, wait: bool = True):
        ev = threading.Event()
        box = {}

        def done(res, err):
            box["res"], box["err"] = res, err
            ev.set()

        ev.box = box  # type: ignore[attr-defined]
        self._q.put((fn, done))
        if not wait:
            return ev
        ev.wait()
        if box.get("err") is not None:
            raise box["err"]
        return box.get("res")

    def _check(self) -> None:
        if self.broken is not None:
            raise KVChannelBroken(f"KV channel broken: {self.broken}")

    def _fail(self, e: BaseException) -> None:
        self.failures += 1
        if isinstance(e, KVTransferTimeout):
            self.broken = str(e)

    # ---------------------------------------------------------------- ops
    def _ctx(self):
        return torch.cuda.stream(self.stream) if self.is_gpu else _Null()

    def send_blocks(self, block_ids: list[int], dst: int,
                    on_done: Optional[Callable[[], None]] = None, wait: bool = False,
                    timeout_s: Optional[float] = None):
        """Pack the blocks (one request's, or several requests' concatenated) and send them
        to rank `dst` (async by default).  `on_done` always runs once the send ended --
        successfully or not -- so the sender's held blocks are never leaked."""
        t_out = self.timeout_s if timeout_s is None else timeout_s

        def fn():
            try:
                self._check()
                with self._ctx():
                    ids = torch.tensor(block_ids, dtype=torch.int32, device=self.device)
                    buf = ops.kv_gather(self.planes, ids)
                    if self.host_staging or not self.is_gpu:
                        if self.is_gpu:
                            self.stream.synchronize()
                        buf = buf.cpu() if self.is_gpu else buf
                    work = dist.isend(buf, dst, group=self.group)
                    _wait(work, t_out, f"KV send of {len(block_ids)} blocks to rank {dst}",
                          self.gloo)
                    if self.is_gpu:
                        self.stream.synchronize()
                self.bytes_sent += buf.numel() * buf.element_size()
                self.transfers += 1
                return True
            except Exception as e:
                self._fail(e)
                print(f"[kv-transfer] send to rank {dst} failed: {e}", flush=True)
                raise
            finally:
                if on_done:
                    on_done()

        return self._submit(fn, wait)

    def gather(self, block_ids: list[int]) -> tuple:
        """Pack blocks NOW on the caller's (compute) stream: later kernels of that stream --
        which may reuse the blocks -- are ordered after the copy, so the caller may free the
        blocks as soon as this returns.  Returns (packed buffer, ready event) for send_packed."""
        ids = torch.tensor(block_ids, dtype=torch.int32, device=self.device)
        buf = ops.kv_gather(self.planes, ids)
        ev = None
        if self.is_gpu:
            ev = torch.cuda.Event()
            ev.record()
        return buf, ev

    def send_packed(self, packed: tuple, dst: int, on_done: Optional[Callable[[], None]] = None,
                    wait: bool = False, timeout_s: Optional[float] = None):
        """Send a buffer packed by gather() (async by default; bounded like send_blocks)."""
        t_out = self.timeout_s if timeout_s is None else timeout_s
        buf, ev = packed

        def fn():
            try:
                self._check()
                with self._ctx():
                    b = buf
                    if self.is_gpu:
                        self.stream.wait_event(ev)
                    if self.host_staging:
                        self.stream.synchronize()
                        b = buf.cpu()
                    work = dist.isend(b, dst, group=self.group)
                    _wait(work, t_out, f"KV send of {buf.shape[1]} blocks to rank {dst}",
                          self.gloo)
                    if self.is_gpu:
                        self.stream.synchronize()
                self.bytes_sent += buf.numel() * buf.element_size()
                self.transfers += 1
                return True
            except Exception as e:
                self._fail(e)
                print(f"[kv-transfer] send to rank {dst} failed: {e}", flush=True)
                raise
            finally:
                if on_done:
                    on_done()

        return self._submit(fn, wait)

    def recv_blocks(self, block_ids: list[int], src: int,
                    timeout_s: Optional[float] = None) -> None:
        """Receive packed KV from rank `src` into our `block_ids` (blocking, bounded)."""
        t_out = self.timeout_s if timeout_s is None else timeout_s

        def fn():
            try:
                self._check()
                with self._ctx():
                    n = len(block_ids)
                    buf = torch.empty(self.planes.shape[0], n, self.block_elems,
                                      dtype=self.kv.dtype, device=self.device)
                    if self.host_staging:
                        hb = torch.empty(buf.shape, dtype=buf.dtype)
                        _wait(dist.irecv(hb, src, group=self.group), t_out,
                              f"KV recv of {n} blocks from rank {src}", True)
                        buf.copy_(hb)
                    else:
                        _wait(dist.irecv(buf, src, group=self.group), t_out,
                              f"KV recv of {n} blocks from rank {src}", self.gloo)
                    ids = torch.tensor(block_ids, dtype=torch.int32, device=self.device)
                    ops.kv_scatter(buf, self.planes, ids)
                    if self.is_gpu:
                        self.stream.synchronize()
                self.bytes_recv += buf.numel() * buf.element_size()
                self.transfers += 1
                return True
            except Exception as e:
                self._fail(e)
                raise

        return self._submit(fn, True)

    def reset(self, generation: int, timeout_s: float = 120.0) -> bool:
        """Rebuild the transfer channel as a NEW process group over the same ranks (every rank
        of the default group must call this with the same generation: P/D pods are 2-rank
        jobs).  Runs on the agent thread, after any queued transfer (which fails fast while
        broken).  Returns True if this call moved the channel to `generation`."""

        if dist.get_world_size() != 2:
            # new_group() completes only when EVERY rank of the default group calls it with
            # this generation; only the 2-rank P/D pod guarantees that (both ends reset)
            raise RuntimeError(f"KV channel reset needs a 2-rank P/D job, world size is "
                               f"{dist.get_world_size()}")

        def fn():
            if generation <= self.generation:
                return False
            ranks = list(range(dist.get_world_size()))
            backend = dist.get_backend(self.group)
            self.group = dist.new_group(ranks=ranks, backend=backend,
                                        timeout=datetime.timedelta(seconds=timeout_s))
            self.gloo = backend == "gloo"
            self.host_staging = self.is_gpu and self.gloo
            self.generation = generation
            self.broken = None
            self.resets += 1
            return True

        return self._submit(fn, True)

    # ---------------------------------------------------------------- hipIpc pull
    def ipc_meta(self) -> dict:
        """What a decode peer needs to map this engine's cache (JSON-able)."""
        import base64

        P, NB, be = self.planes.shape
        return {"blob": base64.b64encode(ops.ipc_export(self.planes)).decode(),
                "planes": int(P), "nblocks": int(NB), "block_elems": int(be),
                "plane_stride": int(self.planes.stride(0))}

    def connect_ipc(self, meta: dict) -> str:
        """Map a prefill peer's cache (once per peer; the mapping lives as long as this agent).
        Returns the peer key for pull(); a decode engine of an N:M pod maps several."""
        import base64

        P, NB, be = self.planes.shape
        if (int(meta["planes"]), int(meta["block_elems"])) != (P, be):
            raise ValueError(f"peer cache geometry {meta['planes']}x{meta['block_elems']} != "
                             f"ours {P}x{be} (same model and block size required)")
        key = meta["blob"]
        if key not in self.peers:
            ptr = ops.ipc_open(base64.b64decode(meta["blob"]), self.device.index)
            self.peers[key] = (ptr, int(meta["nblocks"]), int(meta["plane_stride"]))
        return key

    @property
    def ipc_connected(self) -> bool:
        return bool(self.peers)

    def pull(self, pairs: list, Hkv: int, BS: int, D: int, tail=None,
             tail_jobs: Optional[list] = None, peer: Optional[str] = None) -> float:
        """One kv_pull launch on the agent stream: pairs (peer block, own block) of every
        plane, plus V-tail jobs (peer block, group, count, tail slot); waits for it.  Returns
        the seconds the pull took (host-observed, launch to completion)."""
        if not self.peers:
            raise KVChannelBroken("no peer cache mapped (connect_ipc)")
        if peer is None:
            if len(self.peers) != 1:
                raise ValueError("several peer caches mapped: name the peer")
            peer = next(iter(self.peers))
        ptr, nblocks, stride = self.peers[peer]
        t0 = time.perf_counter()
        with self._ctx():
            ops.kv_pull(ptr, stride, nblocks, self.planes, pairs, Hkv, BS, D, tail=tail,
                        tail_jobs=tail_jobs)
            self.stream.synchronize()
        dt = time.perf_counter() - t0
        self.bytes_recv += self.nbytes(len(pairs))
        self.pull_seconds += dt
        self.transfers += 1
        return dt

    def close(self) -> None:
        if self.peers:
            try:
                torch.cuda.synchronize(self.device)
                for ptr, _, _ in self.peers.values():
                    ops.ipc_close(ptr)
            except Exception:
                pass
            self.peers = {}
        self._q.put(None)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
