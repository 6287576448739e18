"""KV-cache hand-off between a prefill engine and a decode engine (disaggregated P/D).

MI355X design: the prefill and decode engines are two processes (two GPUs of the same
xGMI mesh) in one torch.distributed group (RCCL).  A request's KV cache -- all layers,
K and V, only its own blocks -- is packed by the `kv_gather` HIP kernel into ONE
contiguous buffer [2L, nblk, block_elems] and moved with a single RCCL send/recv (one
large P2P transfer per request instead of 2*L*nblk small ones), then unpacked into the
decode engine's own block ids by `kv_scatter`.  Transfers run on a dedicated stream and
thread on each side, so they overlap both engines' compute.

For Llama-3-8B (32 layers, 8 kv heads x 128, bf16) a 2048-token prompt is 256 MiB of KV:
~2 ms over one xGMI link pair.

Control plane: the decode side asks the prefill server (HTTP POST /kv/push) to send the
blocks of `transfer_id` to its rank, then posts the matching recv.  The same code runs on
CPU with the gloo backend (tests).
"""
from __future__ import annotations

import queue
import threading
from typing import Callable, Optional

import torch
import torch.distributed as dist

from .. import ops


class KVTransferAgent:
    def __init__(self, kv_cache: torch.Tensor, group=None):
        """kv_cache: the engine's [L, 2, NB, block_elems] cache tensor (bf16, or uint8 fp8
        bytes -- moved as bf16 pairs: the copy kernels are dtype-agnostic 16-byte moves)."""
        if kv_cache.dtype == torch.uint8:
            kv_cache = kv_cache.view(torch.bfloat16)
        self.kv = kv_cache
        L, two, NB, be = kv_cache.shape
        self.planes = kv_cache.view(L * two, NB, be)
        self.block_elems = be
        self.group = group
        self.device = kv_cache.device
        self.is_gpu = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.device) if self.is_gpu else None
        self._q: "queue.Queue" = queue.Queue()
        self._thread = threading.Thread(target=self._run, name="kv-transfer", daemon=True)
        self._thread.start()
        self.bytes_sent = 0
        self.bytes_recv = 0
        # gloo moves host tensors only: GPU caches on a gloo group (single-GPU rehearsal of
        # the P/D path) stage through pinned host memory
        self.host_staging = self.is_gpu and dist.is_initialized() and \
            dist.get_backend(group) == "gloo"

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

        self._q.put((fn, done))
        if not wait:
            return ev
        ev.wait()
        if box.get("err") is not None:
            raise box["err"]
        return box.get("res")

    # ---------------------------------------------------------------- ops
    def _ctx(self):
        return torch.cuda.stream(self.stream) if self.is_gpu else _Null()

    def send_blocks(self, block_ids: list[int], dst: int,
                    on_done: Optional[Callable[[], None]] = None, wait: bool = False):
        """Pack the blocks and send them to rank `dst` (async by default)."""

        def fn():
            with self._ctx():
                ids = torch.tensor(block_ids, dtype=torch.int32, device=self.device)
                buf = ops.kv_gather(self.planes, ids)
                if self.host_staging:
                    self.stream.synchronize()
                    dist.send(buf.cpu(), dst, group=self.group)
                else:
                    dist.send(buf, dst, group=self.group)
                if self.is_gpu:
                    self.stream.synchronize()
            self.bytes_sent += buf.numel() * buf.element_size()
            if on_done:
                on_done()
            return True

        return self._submit(fn, wait)

    def recv_blocks(self, block_ids: list[int], src: int) -> None:
        """Receive a packed request KV from rank `src` into our `block_ids` (blocking)."""

        def fn():
            with self._ctx():
                n = len(block_ids)
                buf = torch.empty(self.planes.shape[0], n, self.block_elems, dtype=self.kv.dtype,
                                  device=self.device)
                if self.host_staging:
                    hb = torch.empty(buf.shape, dtype=buf.dtype)
                    dist.recv(hb, src, group=self.group)
                    buf.copy_(hb)
                else:
                    dist.recv(buf, src, group=self.group)
                ids = torch.tensor(block_ids, dtype=torch.int32, device=self.device)
                ops.kv_scatter(buf, self.planes, ids)
                if self.is_gpu:
                    self.stream.synchronize()
            self.bytes_recv += buf.numel() * buf.element_size()
            return True

        return self._submit(fn, True)

    def close(self) -> None:
        self._q.put(None)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
