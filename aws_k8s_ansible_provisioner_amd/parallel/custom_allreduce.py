"""Custom intra-node all-reduce over xGMI peer mappings.

Wraps the one-shot / two-shot HIP kernels of csrc/kernels/custom_allreduce.hip.  Each
TP rank allocates an uncached staging buffer + flag array, exports hipIpc handles, the
handles are all-gathered over torch.distributed, and every rank maps its peers' buffers.
Decode-sized activations (<= ``max_bytes``) then take one kernel launch instead of an
RCCL ring; larger messages (prefill) fall back to RCCL.  The kernels keep their epochs
on the device, so they replay correctly inside captured hipGraphs.

Siblings on the same IPC buffers, flags and device-side epochs: `all_gather` (the
vocab-parallel logits, rank-major column blocks), `broadcast` (rank 0's decode staging
region) and `all_to_all` (the expert-parallel fixed-capacity dispatch and combine).  With all three, a TP decode hipGraph records no RCCL call at all: it replays
across the xGMI mesh and across ranks that share one GPU (gloo control plane) alike.

Policy (xGMI mesh, W ranks): one-shot reads (W-1) x the message over W-1 links at once
and has one flag exchange -- best while the message is small; two-shot moves 2(W-1)/W x
the message with two flag exchanges -- better once link bandwidth, not latency, binds.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from .. import ops

DEFAULT_MAX_BYTES = int(os.environ.get("AKAP_CAR_MAX_BYTES", str(8 << 20)))


def oneshot_limit(world: int) -> int:
    env = os.environ.get("AKAP_CAR_ONESHOT_BYTES")
    if env:
        return int(env)
    return (512 << 10) if world <= 4 else (256 << 10)


def _aligned(t: torch.Tensor) -> bool:
    """The IPC kernels move 16-byte vectors of the user tensor (ops.cpp car_check_aligned)."""
    return t.data_ptr() % 16 == 0


def car_grid(world: int, sharing: int = 1) -> int:
    """Fixed grid of every launch on a communicator: 128 blocks with one rank per GPU; when
    `sharing` ranks run on one physical GPU (the single-GPU rehearsal) they split 128 between
    them, so their spinning blocks leave CUs free for a late peer's GEMMs (AKAP_CAR_BLOCKS)."""
    env = os.environ.get("AKAP_CAR_BLOCKS")
    if env:
        return max(1, min(128, int(env)))
    return max(8, 128 // sharing) if sharing > 1 else 128


def _device_key(device: torch.device) -> str:
    """Physical identity of a GPU: host + PCI domain/bus/device (not the visible index, which
    is 0 in every rank when each rank sees only its own GPU)."""
    import socket

    p = torch.cuda.get_device_properties(device)
    return (f"{socket.gethostname()}:{getattr(p, 'pci_domain_id', 0)}:"
            f"{getattr(p, 'pci_bus_id', 0)}:{getattr(p, 'pci_device_id', 0)}")


def agree_grid(keys: list, grids: list) -> int:
    """Every rank must launch the same fixed grid (the epoch argument in the kernel header):
    the minimum of the ranks' own choices, each made from how many ranks share its physical
    GPU (from the gathered device keys)."""
    share = max(sum(1 for k in keys if k == key) for key in keys)
    auto = max(8, 128 // share) if share > 1 else 128
    return max(1, min(auto, min(grids)))


class CustomAllReduce:
    def __init__(self, group=None, device: Optional[torch.device] = None,
                 max_bytes: int = DEFAULT_MAX_BYTES, buffer_bytes: int = 0):
        """max_bytes: all-reduce policy threshold (larger messages go to RCCL); buffer_bytes:
        staging capacity, raised above max_bytes so the all-gather of a decode step's
        vocab-parallel logits (rows x vocab/tp) and the step broadcast always fit -- a decode
        hipGraph then never falls back to a process-group collective."""
        ops.load_native(required=True)
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.max_bytes = max_bytes
        self.buffer_bytes = max(max_bytes, buffer_bytes)
        self.oneshot_bytes = oneshot_limit(self.world)
        max_elems = (self.buffer_bytes // 2 + 7) // 8 * 8
        # one grid for the whole communicator: gathered device identities decide sharing, and
        # the ranks take the minimum (a rank with a different env or visibility cannot leave
        # the others waiting on flags its smaller grid never sets)
        info: list = [None] * self.world
        env = os.environ.get("AKAP_CAR_BLOCKS")
        dist.all_gather_object(info, (_device_key(self.device),
                                      max(1, min(128, int(env))) if env else 128),
                               group=group)
        self.blocks = agree_grid([k for k, _ in info], [g for _, g in info])
        self.h = torch.ops.akap.car_create(self.device.index, self.rank, self.world, max_elems,
                                           self.blocks)
        mine = torch.ops.akap.car_ipc_handles(self.h)
        allh: list = [None] * self.world
        dist.all_gather_object(allh, mine.numpy().tobytes(), group=group)
        handles = torch.stack([torch.frombuffer(bytearray(b), dtype=torch.uint8).view(2, -1)
                               for b in allh])
        torch.ops.akap.car_open(self.h, handles)
        # the kernels' sticky timeout word (device int32): replayed decode steps copy it to
        # pinned host memory and the runner checks it before emitting tokens
        self.err_word = torch.ops.akap.car_error_word(self.h)
        dist.barrier(group=group)

    def should_use(self, x: torch.Tensor) -> bool:
        nbytes = x.numel() * x.element_size()
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous()
                and x.numel() % 8 == 0 and nbytes <= self.max_bytes and _aligned(x))

    def all_reduce(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        out = x if out is None else out
        two = x.numel() * 2 > self.oneshot_bytes and self.world > 2
        torch.ops.akap.car_all_reduce(self.h, x, out, two)
        return out

    def all_reduce_resnorm(self, x: torch.Tensor, residual: torch.Tensor, ln: torch.Tensor,
                           a_out: torch.Tensor, ss: torch.Tensor) -> None:
        """x = this rank's row-parallel partial sums [M, d]; after the exchange every rank has
        residual += sum, a_out = residual * ln, ss += row sums of residual^2 (the decode
        chain's residual-add epilogue, fused into the all-reduce's store pass)."""
        two = x.numel() * 2 > self.oneshot_bytes and self.world > 2
        torch.ops.akap.car_all_reduce_resnorm(self.h, x, residual, ln, a_out, ss, two)

    def gather_ok(self, x: torch.Tensor) -> bool:
        nbytes = x.numel() * x.element_size()
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous()
                and x.numel() % 8 == 0 and nbytes <= self.buffer_bytes and x.dim() >= 1
                and x.shape[-1] % 8 == 0 and _aligned(x))

    def all_gather(self, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """x [R, n] (this rank's shard) -> out [R, world*n], rank-major column blocks."""
        torch.ops.akap.car_all_gather(self.h, x, out)
        return out

    def a2a_ok(self, x: torch.Tensor) -> bool:
        nbytes = x.numel() * x.element_size()
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous()
                and x.numel() % (8 * self.world) == 0 and nbytes <= self.buffer_bytes
                and _aligned(x))

    def all_to_all(self, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """Equal segments: x [world * seg] (segment d to rank d) -> out (segment p from rank p)."""
        torch.ops.akap.car_all_to_all(self.h, x, out)
        return out

    def bcast_ok(self, t: torch.Tensor) -> bool:
        nbytes = t.numel() * t.element_size()
        return (t.is_cuda and t.is_contiguous() and nbytes % 16 == 0
                and nbytes <= self.buffer_bytes and _aligned(t))

    def broadcast(self, t: torch.Tensor, root: int) -> torch.Tensor:
        """In place: every rank's t becomes group rank `root`'s t."""
        torch.ops.akap.car_broadcast(self.h, t, root)
        return t

    def error(self) -> int:
        return int(torch.ops.akap.car_error(self.h))

    def close(self) -> None:
        if self.h is not None:
            torch.ops.akap.car_destroy(self.h)
            self.h = None
