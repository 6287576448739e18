"""Collectives used by the model (TP / EP / P-D) on RCCL over xGMI.

MI355X nodes are a fully-connected xGMI mesh (7 links x ~153 GB/s per GPU), not a
switch: a ring all-reduce is bound by one link per hop.  The policy here:
  * decode-time all-reduces (a few KB-MB per layer) -> the custom one-/two-shot xGMI
    kernel (parallel/custom_allreduce.py, one launch, graph-capturable); larger ones
    (prefill) -> one RCCL all_reduce in place;
  * vocab-parallel logits -> the custom IPC all-gather (decode sizes; rank-major columns
    straight into the pre-allocated result) or one RCCL all_gather;
  * the TP decode step's input region -> the custom IPC broadcast (or RCCL broadcast);
  * MoE token dispatch/combine -> the custom IPC all-to-all (fixed-capacity decode steps,
    equal splits) or all_to_all_single with explicit split sizes;
  * KV hand-off (P/D) -> one packed send/recv per request (see parallel/kv_transfer.py).
All functions are no-ops for a group of size 1, so single-GPU code paths pay nothing.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .state import get_state


def tp_all_reduce(x: torch.Tensor) -> torch.Tensor:
    st = get_state()
    if st.tp_size == 1:
        return x
    if st.car is not None and st.car.should_use(x):
        return st.car.all_reduce(x)
    if st.car is not None and st.backend == "gloo" and _car_pieces_ok(x, st.car):
        # ranks sharing one GPU over a gloo control plane (single-GPU rehearsal): prefill-sized
        # all-reduces stay on the device in max_bytes pieces of the IPC kernel instead of a
        # host-staged gloo all-reduce
        flat = x.view(-1)
        cap = st.car.max_bytes // x.element_size() // 8 * 8
        pieces = -(-flat.numel() // cap)
        per = -(-flat.numel() // pieces)
        step = (per + 7) // 8 * 8  # near-equal pieces, each 16-B aligned
        for i in range(0, flat.numel(), step):
            st.car.all_reduce(flat[i:i + step])
        # a piece whose flag wait timed out only raises the kernel's error word: the step
        # checks it once at its end (check_deferred), not a device sync per all-reduce
        _UNCHECKED[0] = True
        return x
    dist.all_reduce(x, group=st.tp_group)
    return x


_UNCHECKED = [False]  # a piecewise / chunked IPC collective ran since the last check


class CollectiveTimeout(RuntimeError):
    """A custom IPC collective gave up waiting for a peer (its bounded flag wait expired):
    the step summed stale staging, so its outputs must not be used.  The kernels' error word
    is sticky, so every later step fails too: the engine reports unhealthy and is restarted
    (device-side epochs cannot be realigned across ranks without one)."""


def check_deferred() -> None:
    """End of an eager step: raise if one of its piecewise IPC collectives timed out (the
    kernels only set an error word; silently summing on would corrupt the step)."""
    if not _UNCHECKED[0]:
        return
    _UNCHECKED[0] = False
    st = get_state()
    if st is not None and st.car is not None and st.car.error():
        raise CollectiveTimeout("custom IPC collective timed out in a piecewise prefill step")


def _car_pieces_ok(x: torch.Tensor, car) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous()
            and x.numel() % 8 == 0 and car.max_bytes >= 4096)


def tp_all_reduce_resnorm(partial: torch.Tensor, residual: torch.Tensor, ln: torch.Tensor,
                          a_out: torch.Tensor, ss: torch.Tensor) -> None:
    """Row-parallel partial sums -> the decode chain's residual epilogue on every TP rank:
    residual += all_reduce(partial); a_out = residual * ln; ss += row sums of residual^2
    (the next RMSNorm's row scale is applied by the consumer GEMM, dgemm ss_in).  Decode
    sizes take the custom xGMI all-reduce with this epilogue fused into its store pass (one
    launch); otherwise RCCL all_reduce + the same elementwise math."""
    st = get_state()
    if st.tp_size > 1 and st.car is not None and st.car.should_use(partial) and \
            ln.numel() % 512 == 0:
        st.car.all_reduce_resnorm(partial, residual, ln, a_out, ss)
        return
    if st.tp_size > 1:
        # no fused epilogue for this row width: the plain custom all-reduce (still one of our
        # capturable kernels) or RCCL, then the elementwise epilogue
        tp_all_reduce(partial)
    r = (partial.float() + residual.float()).to(residual.dtype)
    residual.copy_(r)
    a_out.copy_((r.float() * ln.float()).to(a_out.dtype))
    ss[: r.shape[0]] += r.float().pow(2).sum(-1)


_GATHER_WS: dict = {}
_GATHER_OLD: list = []  # outgrown workspaces stay alive: captured hipGraphs may address them


def _gather_ws(key: str, rows: int, cols: int, dtype, device) -> torch.Tensor:
    """Persistent gather workspace (grown, never shrunk): the per-step logits gather reuses
    one allocation instead of asking the allocator for [tp*B, V/tp] + [B, V] every step."""
    k = (key, cols, dtype, str(device))
    buf = _GATHER_WS.get(k)
    if buf is None or buf.shape[0] < rows:
        if buf is not None:
            _GATHER_OLD.append(buf)
        buf = torch.empty(rows, cols, dtype=dtype, device=device)
        _GATHER_WS[k] = buf
    return buf[:rows]


def tp_all_gather_last(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Gather shards along the last dim: [.., n] x tp -> [.., n*tp].  One all_gather into a
    single preallocated [tp, .., n] buffer (no per-rank tensor list) + one transposing copy
    into a preallocated result (or `out`)."""
    st = get_state()
    if st.tp_size == 1:
        return x
    x = x.contiguous()
    flat = x.reshape(1, -1) if x.dim() == 1 else x.reshape(-1, x.shape[-1])
    R, n = flat.shape
    if st.car is not None and st.car.gather_ok(flat):
        if out is None:
            out = _gather_ws("result", R, st.tp_size * n, x.dtype, x.device)
        st.car.all_gather(flat, out.view(R, st.tp_size * n))
        return out.view(*x.shape[:-1], st.tp_size * n)
    buf = _gather_ws("gather", st.tp_size * R, n, x.dtype, x.device)
    dist.all_gather_into_tensor(buf, flat, group=st.tp_group)  # rank-major rows
    if out is None:
        out = _gather_ws("result", R, st.tp_size * n, x.dtype, x.device)
    out.view(R, st.tp_size, n).copy_(buf.view(st.tp_size, R, n).transpose(0, 1))
    return out.view(*x.shape[:-1], st.tp_size * n)


def tp_all_gather_rows(out: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """Concatenate every TP rank's x along dim 0 into out (rank order): the IPC all-gather of
    the flattened rows when it fits (capturable on any control backend), else RCCL."""
    st = get_state()
    flat = x.contiguous().view(1, -1)
    if st.car is not None and st.car.gather_ok(flat) and out.is_contiguous():
        st.car.all_gather(flat, out.view(1, -1))
        return out
    if (st.car is not None and st.backend == "gloo" and x.dim() == 2 and out.is_contiguous()
            and _car_pieces_ok(x.contiguous(), st.car) and x.shape[1] % 8 == 0):
        # ranks sharing one GPU over a gloo control plane (single-GPU rehearsal of an EP x TP
        # prefill): row slabs through the IPC all-gather instead of a host-staged gloo gather
        W, (per, d) = st.tp_size, x.shape
        rows = max(1, st.car.buffer_bytes // (2 * d))  # the staged shard fits the buffer
        xc, dst = x.contiguous(), out.view(W, per, d)
        for r0 in range(0, per, rows):
            r1 = min(per, r0 + rows)
            piece = xc[r0:r1].reshape(1, -1)
            tmp = torch.empty(1, W * piece.numel(), dtype=x.dtype, device=x.device)
            st.car.all_gather(piece, tmp)
            dst[:, r0:r1].copy_(tmp.view(W, r1 - r0, d))
        _UNCHECKED[0] = True
        return out
    dist.all_gather_into_tensor(out, x.contiguous(), group=st.tp_group)
    return out


def ep_chunk_rows(C: int, D: int, x: torch.Tensor) -> int:
    """Rows per destination per chunk of a fixed-capacity EP exchange of [W, C, D] rows: C
    (one exchange) unless the message outgrows the IPC staging on a single-GPU gloo
    rehearsal, where it runs as chunks of [W, R, D] contiguous blocks (MoEBlock._ep_fixed lays
    the rows out chunk-major, so no slab copies are needed)."""
    st = get_state()
    if (st is None or st.car is None or st.tp_size != st.world_size or not x.is_cuda
            or x.dtype != torch.bfloat16 or D % 8):
        return C
    W = st.world_size
    if W * C * D * 2 <= st.car.buffer_bytes or st.backend != "gloo":
        return C  # one IPC launch, or RCCL all_to_all_single on a node
    R = max(8, st.car.buffer_bytes // (2 * D * W) // 8 * 8)
    return min(C, R)


def ep_all_to_all_equal(recv: torch.Tensor, send: torch.Tensor, chunks: int = 1
                        ) -> torch.Tensor:
    """All-to-all over the whole job with equal splits (the fixed-capacity EP dispatch /
    combine): the custom IPC kernel when the TP group is the whole job and the message fits
    its staging (capturable on any control backend), else all_to_all_single.  chunks > 1: the
    rows are chunk-major ([chunks, W, R, D], ep_chunk_rows) and every chunk is one IPC launch."""
    st = get_state()
    if chunks > 1:
        s2, r2 = send.view(chunks, -1), recv.view(chunks, -1)
        for k in range(chunks):
            st.car.all_to_all(s2[k], r2[k])
        _UNCHECKED[0] = True
        return recv
    if (st.car is not None and st.tp_size == st.world_size and st.car.a2a_ok(send)
            and recv.is_contiguous() and recv.dtype == send.dtype):
        return st.car.all_to_all(send.view(-1), recv.view(-1)).view_as(recv)
    dist.all_to_all_single(recv, send)
    return recv


def tp_broadcast(t: torch.Tensor) -> torch.Tensor:
    """In place: every TP rank's t becomes the TP group's rank-0 copy (the custom IPC
    broadcast when it fits -- capturable on any control backend -- else RCCL)."""
    st = get_state()
    if st.tp_size == 1:
        return t
    if st.car is not None and st.car.bcast_ok(t):
        return st.car.broadcast(t, 0)
    dist.broadcast(t, src=st.rank - st.tp_rank, group=st.tp_group)
    return t


def all_to_all(x: torch.Tensor, out_splits: list[int], in_splits: list[int], group=None
               ) -> torch.Tensor:
    out = x.new_empty((sum(out_splits),) + tuple(x.shape[1:]))
    dist.all_to_all_single(out, x.contiguous(), out_splits, in_splits, group=group)
    return out


def tp_all_true(flag: bool) -> bool:
    """True on every TP rank iff it is True on all of them (MIN all-reduce of a flag): for
    per-rank decisions that must agree before a collective-issuing code path runs."""
    st = get_state()
    if st.tp_size == 1 or st.tp_group is None:
        return bool(flag)
    dev = "cuda" if dist.get_backend(st.tp_group) == "nccl" else "cpu"
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=st.tp_group)
    return bool(t.item())


def broadcast_object(obj, src: int = 0, group=None):
    st = get_state()
    if st.world_size == 1:
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src, group=group)
    return lst[0]
