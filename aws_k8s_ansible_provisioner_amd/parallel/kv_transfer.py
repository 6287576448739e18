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


class KVIpcOpenTimeout(KVChannelBroken):
    """hipIpcOpenMemHandle of a peer cache did not return in time (the caller falls back to
    the p2p transport for that peer)."""


IPC_OPEN_TIMEOUT_S = float(os.environ.get("AKAP_IPC_OPEN_TIMEOUT_S", "60"))


def bounded_call(fn: Callable, timeout_s: float, what: str):
    """Run fn() on a daemon thread and wait at most timeout_s: a driver call that never
    returns (hipIpcOpenMemHandle of a large export on a shared device) leaves that thread
    parked but never blocks the caller -- a server thread, a handshake -- forever."""
    box: dict = {}

    def run():
        try:
            box["v"] = fn()
        except BaseException as e:  # surfaced to the caller
            box["e"] = e

    t = threading.Thread(target=run, name="kv-ipc-open", daemon=True)
    t.start()
    t.join(timeout_s)
    if t.is_alive():
        raise KVIpcOpenTimeout(f"{what} did not return within {timeout_s:.0f}s")
    if "e" in box:
        raise box["e"]
    return box["v"]


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
    def __init__(self, kv_cache: torch.Tensor, group=None, timeout_s: float = DEFAULT_TIMEOUT_S,
                 pair=None):
        """kv_cache: the engine's [L, 2, NB, block_elems] cache tensor (bf16, or uint8 fp8
        bytes -- moved as bf16 pairs: the copy kernels are dtype-agnostic 16-byte moves).
        pair: (ProcessGroup, backend name) of a two-rank channel between two independently
        started servers (two-pod P/D, `connect_pair` / `PairHost`) -- used instead of a
        group of the default torch.distributed world."""
        # the cache is one tensor [L, 2, NB, be] or its layer-range segments (one allocation
        # each: model_runner.kv_segs); planes are addressed per segment
        segs = list(kv_cache) if isinstance(kv_cache, (list, tuple)) else [kv_cache]
        # fp8: bytes moved as bf16 pairs; kv_pull takes the halved block (ops.cpp), and an fp8
        # cache has no V tail
        self.byte_cache = segs[0].dtype == torch.uint8
        if self.byte_cache:
            segs = [t.view(torch.bfloat16) for t in segs]
        self.segs = segs
        self.kv = segs[0]
        self.planes_list = [t.view(t.shape[0] * t.shape[1], t.shape[2], t.shape[3]) for t in segs]
        self.planes = self.planes_list[0]
        self.num_planes = sum(p.shape[0] for p in self.planes_list)
        self.nblocks = segs[0].shape[2]
        be = segs[0].shape[3]
        self.block_elems = be
        self.group = group
        self.timeout_s = timeout_s
        self.device = segs[0].device
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
        self.pg = pair[0] if pair is not None else None
        if pair is not None:
            self.gloo = pair[1] == "gloo"
        else:
            self.gloo = dist.is_initialized() and dist.get_backend(group) == "gloo"
        self.host_staging = self.is_gpu and self.gloo
        self.peers: dict = {}  # hipIpc: peer key -> (mapped cache address, blocks, plane stride)
        self.ipc_failed: dict = {}  # peer key -> why its mapping failed (-> p2p for that peer)
        self.ipc_open_timeout_s = IPC_OPEN_TIMEOUT_S
        self.pull_seconds = 0.0

    def _ids(self, block_ids) -> torch.Tensor:
        """Block ids as a device tensor, range-checked on the host first: the gather / scatter
        kernels index the cache with them unchecked, so an id outside [0, nblocks) (e.g. from
        a malformed control message) would read or write past the cache."""
        ids = [int(b) for b in block_ids]
        bad = [b for b in ids if not 0 <= b < self.nblocks]
        if bad:
            raise IndexError(f"KV block ids {bad[:8]} outside the cache's {self.nblocks} blocks")
        return torch.tensor(ids, dtype=torch.int32, device=self.device)

    def probe_channel(self, rank: int, peer: str, nbytes: int, log=print) -> Optional[dict]:
        """Time one `nbytes` transfer over this pair channel (rank 0 sends, rank 1 receives),
        right after the channel formed and before any KV moves on it: the achieved GB/s and
        RCCL's chosen transport go to CHANNEL_PROBES[peer] (and /metrics), so a deployment
        sees what its prefill -> decode path really is (xGMI peer-to-peer vs host-staged)."""
        if nbytes <= 0 or self.pg is None:
            return None
        on_dev = self.is_gpu and not self.gloo
        dev = self.device if on_dev else torch.device("cpu")
        buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        op = self._isend if rank == 0 else self._irecv
        other = 1 - rank
        what = f"KV channel probe with {peer}"
        with self._ctx():
            _wait(op(buf[: 1 << 20], other), self.timeout_s, what, self.gloo)  # connect + sync
            if on_dev:
                self.stream.synchronize()
            t0 = time.perf_counter()
            _wait(op(buf, other), self.timeout_s, what, self.gloo)
            if on_dev:
                self.stream.synchronize()
            dt = time.perf_counter() - t0
        backend = "gloo" if self.gloo else "nccl"
        res = {"gbps": nbytes / dt / 1e9, "bytes": nbytes, "seconds": dt,
               "transport": channel_transport(backend), "role": "send" if rank == 0 else "recv"}
        CHANNEL_PROBES[peer] = res
        log(f"[pd] KV channel probe {peer}: {nbytes / 2**20:.0f} MiB in {dt * 1e3:.1f} ms = "
            f"{res['gbps']:.2f} GB/s over {res['transport']} ({backend})")
        return res

    def nbytes(self, nblk: int) -> int:
        return self.num_planes * nblk * self.block_elems * self.kv.element_size()

    def _gather(self, ids: torch.Tensor) -> torch.Tensor:
        """Pack blocks `ids` of every plane (all segments) into [planes, n, block_elems]."""
        if len(self.planes_list) == 1:
            return ops.kv_gather(self.planes, ids)
        return torch.cat([ops.kv_gather(pl, ids) for pl in self.planes_list], 0)

    def _scatter(self, buf: torch.Tensor, ids: torch.Tensor) -> None:
        p0 = 0
        for pl in self.planes_list:
            ops.kv_scatter(buf[p0:p0 + pl.shape[0]], pl, ids)
            p0 += pl.shape[0]

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
    def _isend(self, buf: torch.Tensor, dst: int):
        if self.pg is not None:
            return self.pg.send([buf], dst, 0)
        return dist.isend(buf, dst, group=self.group)

    def _irecv(self, buf: torch.Tensor, src: int):
        if self.pg is not None:
            return self.pg.recv([buf], src, 0)
        return dist.irecv(buf, src, group=self.group)

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
                    ids = self._ids(block_ids)
                    buf = self._gather(ids)
                    if self.host_staging or not self.is_gpu:
                        if self.is_gpu:
                            self.stream.synchronize()
                        buf = buf.cpu() if self.is_gpu else buf
                    work = self._isend(buf, dst)
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
        ids = self._ids(block_ids)
        buf = self._gather(ids)
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
                    work = self._isend(b, dst)
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
                    buf = torch.empty(self.num_planes, n, self.block_elems,
                                      dtype=self.kv.dtype, device=self.device)
                    if self.host_staging:
                        hb = torch.empty(buf.shape, dtype=buf.dtype)
                        _wait(self._irecv(hb, src), t_out,
                              f"KV recv of {n} blocks from rank {src}", True)
                        buf.copy_(hb)
                    else:
                        _wait(self._irecv(buf, src), t_out,
                              f"KV recv of {n} blocks from rank {src}", self.gloo)
                    ids = self._ids(block_ids)
                    self._scatter(buf, ids)
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

        if self.pg is not None:
            raise RuntimeError("a pair channel is rebuilt by a new connect_pair (generation + 1)")
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
        """What a decode peer needs to map this engine's cache (JSON-able): one hipIpc export
        per cache segment (allocation) and the geometry."""
        import base64

        return {"segments": [{"blob": base64.b64encode(ops.ipc_export(pl)).decode(),
                              "planes": int(pl.shape[0])} for pl in self.planes_list],
                "planes": int(self.num_planes), "nblocks": int(self.nblocks),
                "block_elems": int(self.block_elems),
                "plane_stride": int(self.planes.stride(0))}

    def connect_ipc(self, meta: dict) -> str:
        """Map a prefill peer's cache segments (once per peer; the mappings live as long as
        this agent), each open bounded by AKAP_IPC_OPEN_TIMEOUT_S.  Returns the peer key for
        pull(); a decode engine of an N:M pod maps several peers."""
        import base64

        if (int(meta["planes"]), int(meta["block_elems"])) != (self.num_planes, self.block_elems):
            raise ValueError(f"peer cache geometry {meta['planes']}x{meta['block_elems']} != "
                             f"ours {self.num_planes}x{self.block_elems} (same model and block "
                             f"size required)")
        segs = meta["segments"]
        key = segs[0]["blob"]
        if key in self.ipc_failed:
            raise KVIpcOpenTimeout(self.ipc_failed[key])
        if key not in self.peers:
            dev = self.device.index
            stride = int(meta["plane_stride"]) * self.kv.element_size()
            ptrs, table = [], []
            try:
                for sg in segs:
                    blob = base64.b64decode(sg["blob"])
                    ptr = bounded_call(lambda: ops.ipc_open(blob, dev), self.ipc_open_timeout_s,
                                       f"hipIpc mapping of a {sg['planes']}-plane peer cache "
                                       f"segment")
                    ptrs.append(ptr)
                    table += [ptr + i * stride for i in range(int(sg["planes"]))]
            except KVIpcOpenTimeout as e:
                self.ipc_failed[key] = str(e)
                print(f"[kv-transfer] {e}: this peer falls back to the p2p transport",
                      flush=True)
                raise
            self.peers[key] = (table, int(meta["nblocks"]), ptrs)
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
        table, nblocks, _ = self.peers[peer]
        if self.byte_cache and tail_jobs:
            raise ValueError("V-tail jobs with an fp8 KV cache (fp8 caches have no V tail)")
        t0 = time.perf_counter()
        with self._ctx():
            ops.kv_pull(table, nblocks, self.planes_list, pairs, Hkv, BS, D, tail=tail,
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
                for _, _, ptrs in self.peers.values():
                    for ptr in ptrs:
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


# ------------------------------------------------------------------------------ two-pod P/D
# Prefill and decode servers started independently (separate Deployments / pods, no shared
# launcher or MASTER_ADDR) bootstrap a KV channel per (decode peer, generation) over HTTP:
# the decode server POSTs /kv/hello {peer, generation} to the prefill server, which answers
# with the port of its TCPStore and joins a fresh two-rank process group (prefill rank 0,
# decode rank 1) under the prefix "<peer>/<generation>" while the decode server joins the same
# group as a store client.  A broken channel is replaced by a hello at generation + 1.  The
# hipIpc pull needs no channel at all (/kv/lease carries the export handle); this channel
# carries the p2p transport (and the p2p fallback of a peer whose cache cannot be mapped).

# peer -> the channel probe's result ({"gbps", "bytes", "seconds", "transport", "role"}): what
# a freshly formed pair channel actually moves, exported as akap:kv_channel_probe_gbps
CHANNEL_PROBES: dict = {}


def probe_bytes(gpu: bool) -> int:
    """Size of the channel probe (AKAP_PD_PROBE_MIB; 0 disables): 256 MiB between GPU
    engines -- large enough that link bandwidth, not latency, sets the rate -- 8 MiB on CPU."""
    env = os.environ.get("AKAP_PD_PROBE_MIB")
    mib = float(env) if env else (256.0 if gpu else 8.0)
    return int(mib * 2**20)


def transport_from_rccl_log(text: str) -> str:
    """RCCL's transport for a connection, from its INFO log (NCCL_DEBUG=INFO with the P2P /
    SHM / NET subsystems): "P2P" (peer mapping: xGMI / PCIe peer-to-peer), "SHM" (host shared
    memory), "NET" (sockets / IB: what two pods that see neither each other's GPU nor a common
    /dev/shm end up on), else "unknown"."""
    seen = set()
    for line in text.splitlines():
        if " via " not in line:
            continue
        via = line.split(" via ", 1)[1].strip()
        for kind in ("P2P", "SHM", "NET"):
            if via.startswith(kind):
                seen.add(kind)
    for kind in ("NET", "SHM", "P2P"):  # the slowest path any channel took
        if kind in seen:
            return kind
    return "unknown"


def channel_transport(backend: str) -> str:
    if backend == "gloo":
        return "gloo-tcp"
    path = os.environ.get("NCCL_DEBUG_FILE")
    if not path:
        return "unknown"
    import socket

    path = path.replace("%h", socket.gethostname()).replace("%p", str(os.getpid()))
    try:
        with open(path, errors="replace") as f:
            return transport_from_rccl_log(f.read())
    except OSError:
        return "unknown"


def enable_rccl_transport_log() -> None:
    """Before the first RCCL communicator of this process: have RCCL log its connection
    transports to a per-process file (unless the operator configured NCCL_DEBUG already), so
    the channel probe can report which one the pair channel got."""
    if "NCCL_DEBUG" in os.environ:
        return
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT,P2P,SHM,NET")
    os.environ.setdefault("NCCL_DEBUG_FILE", "/tmp/akap-rccl.%h.%p.log")


def pair_backend(kv: torch.Tensor) -> str:
    """gloo on CPU caches (and AKAP_PD_PAIR_BACKEND=gloo: host-staged, works between pods that
    see no common device), RCCL between GPU engines."""
    env = os.environ.get("AKAP_PD_PAIR_BACKEND")
    if env in ("gloo", "nccl"):
        return env
    return "nccl" if kv.is_cuda else "gloo"


def _pair_group(store, prefix: str, rank: int, backend: str, timeout_s: float, device=None):
    ps = dist.PrefixStore(prefix, store)
    to = datetime.timedelta(seconds=timeout_s)
    if backend == "gloo":
        return dist.ProcessGroupGloo(ps, rank, 2, to)
    opts = dist.ProcessGroupNCCL.Options()
    opts._timeout = to
    return dist.ProcessGroupNCCL(ps, rank, 2, opts)


class PairHost:
    """Prefill side of the two-pod bootstrap: a TCPStore server on `port` and the pair agents
    formed so far (peer id -> KVTransferAgent)."""

    def __init__(self, kv: torch.Tensor, port: int, timeout_s: float = DEFAULT_TIMEOUT_S):
        self.kv = kv
        self.timeout_s = timeout_s
        self.store = dist.TCPStore("0.0.0.0", port, None, True,
                                   datetime.timedelta(seconds=max(timeout_s, 60.0)),
                                   wait_for_workers=False)
        self.port = self.store.port
        self.agents: dict = {}
        self.errors: dict = {}
        self.lock = threading.Lock()

    def accept(self, peer: str, generation: int, backend: str) -> str:
        """Join the pair group for (peer, generation) in the background; returns the prefix."""
        prefix = f"akap-pair/{peer}/{int(generation)}"

        def form():
            try:
                pg = _pair_group(self.store, prefix, 0, backend, self.timeout_s)
                ag = KVTransferAgent(self.kv, timeout_s=self.timeout_s, pair=(pg, backend))
                ag.generation = int(generation)
                # the decode side receives this right after joining; registered only after
                # it, so no KV send can interleave with the probe on the channel
                ag.probe_channel(0, peer, probe_bytes(ag.is_gpu))
                with self.lock:
                    old = self.agents.get(peer)
                    self.agents[peer] = ag
                    self.errors.pop(peer, None)
                if old is not None:
                    old.close()
            except Exception as e:  # the decode side times out and retries with a new hello
                with self.lock:
                    self.errors[peer] = repr(e)

        threading.Thread(target=form, name=f"kv-pair-{peer}", daemon=True).start()
        return prefix

    def agent(self, peer: str, wait_s: float = 10.0) -> Optional["KVTransferAgent"]:
        """The pair agent of `peer` (waits briefly: the decode side may return from the group
        rendezvous a moment before this side registers it)."""
        deadline = time.monotonic() + wait_s
        while True:
            with self.lock:
                ag = self.agents.get(peer)
            if ag is not None or time.monotonic() > deadline:
                return ag
            time.sleep(0.01)


def connect_pair(kv: torch.Tensor, host: str, port: int, prefix: str, backend: str,
                 timeout_s: float = DEFAULT_TIMEOUT_S) -> "KVTransferAgent":
    """Decode side of the two-pod bootstrap: join the pair group the prefill server opened for
    us (rank 1) and return an agent on it."""
    store = dist.TCPStore(host, int(port), None, False,
                          datetime.timedelta(seconds=max(timeout_s, 60.0)))
    pg = _pair_group(store, prefix, 1, backend, timeout_s)
    ag = KVTransferAgent(kv, timeout_s=timeout_s, pair=(pg, backend))
    ag._store = store  # keep the client alive with the group
    ag.probe_channel(1, f"{host}:{port}", probe_bytes(ag.is_gpu))
    return ag
