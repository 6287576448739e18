"""Process-group state: one process per GPU, torch.distributed over RCCL ("nccl" on ROCm).

Groups:
  * world  -- every engine rank of this job
  * tp     -- tensor-parallel group (contiguous ranks: TP stays inside one node's xGMI mesh)
  * dp     -- ranks with the same tp rank (replica / expert-parallel axis)

On CPU (tests) the same code runs on the gloo backend.
"""
from __future__ import annotations

import dataclasses
import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


@dataclasses.dataclass
class ParallelState:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    tp_size: int = 1
    tp_rank: int = 0
    dp_size: int = 1
    dp_rank: int = 0
    tp_group: Optional[object] = None
    dp_group: Optional[object] = None
    backend: str = "none"
    car: Optional[object] = None   # CustomAllReduce over the TP group (xGMI peer mappings)

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1


_STATE = ParallelState()


def get_state() -> ParallelState:
    return _STATE


def env_rank_info() -> tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init_distributed(tp_size: int = 1, backend: Optional[str] = None,
                     device: Optional[str] = None, timeout_s: int = 600,
                     car_buffer_bytes: int = 0) -> ParallelState:
    """Initialise torch.distributed from torchrun env vars and build TP/DP groups.

    backend: "nccl" (RCCL over xGMI on MI355X) when GPUs are present, else "gloo".
    """
    global _STATE
    rank, world, local = env_rank_info()
    if torch.cuda.is_available():
        # more ranks than devices only in single-GPU rehearsals (gloo): share the device
        local = local % max(1, torch.cuda.device_count())
    if backend is None:
        # an already initialised default group (bench.py, tests) decides: its collectives are
        # what tp_all_reduce falls back to
        if dist.is_initialized():
            backend = dist.get_backend()
        else:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend == "nccl":
            torch.cuda.set_device(local)
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(**kw)
    elif backend == "nccl" and torch.cuda.is_available():
        torch.cuda.set_device(local)
    if world % tp_size != 0:
        raise ValueError(f"world size {world} not divisible by tp {tp_size}")
    st = ParallelState(rank=rank, world_size=world, local_rank=local, tp_size=tp_size,
                       tp_rank=rank % tp_size, dp_size=world // tp_size, dp_rank=rank // tp_size,
                       backend=backend if world > 1 else "none")
    if world > 1:
        for g in range(world // tp_size):
            ranks = list(range(g * tp_size, (g + 1) * tp_size))
            grp = dist.new_group(ranks)
            if rank in ranks:
                st.tp_group = grp
        for t in range(tp_size):
            ranks = list(range(t, world, tp_size))
            grp = dist.new_group(ranks)
            if rank in ranks:
                st.dp_group = grp
    # the custom all-reduce rides on RCCL ranks; AKAP_CUSTOM_AR_GLOO=1 also builds it for gloo
    # ranks that share one GPU (single-GPU rehearsal: the IPC mappings work within a device)
    car_gloo = (backend == "gloo" and torch.cuda.is_available()
                and os.environ.get("AKAP_CUSTOM_AR_GLOO") == "1")
    if (world > 1 and tp_size > 1 and (backend == "nccl" or car_gloo)
            and os.environ.get("AKAP_CUSTOM_AR", "1") != "0"):
        from .custom_allreduce import CustomAllReduce
        st.car = CustomAllReduce(group=st.tp_group, device=torch.device("cuda", local),
                                 buffer_bytes=car_buffer_bytes)
    _STATE = st
    return st


def set_state(st: ParallelState) -> None:
    global _STATE
    _STATE = st


def drain_pending_collectives(st: Optional[ParallelState] = None) -> None:
    """Block until the RCCL watchdog has retired every outstanding work of our groups.

    Call before a hipGraph capture that records collectives: the watchdog polls each pending
    work's end event, and on ROCm querying an event whose stream has since joined a capture
    fails with hipErrorCapturedEvent, which terminates the process from the watchdog thread.
    The warm-up collectives issued just before capture are exactly such works."""
    if not dist.is_initialized():
        return
    st = st or _STATE
    seen = set()
    for grp in (dist.group.WORLD, st.tp_group, st.dp_group):
        if grp is None or id(grp) in seen:
            continue
        seen.add(id(grp))
        try:
            if dist.get_backend(grp) != "nccl":
                continue
            grp._wait_for_pending_works()
        except (RuntimeError, NotImplementedError, AttributeError, ValueError):
            pass


def destroy() -> None:
    global _STATE
    if _STATE.car is not None:
        _STATE.car.close()
    if dist.is_initialized():
        dist.destroy_process_group()
    _STATE = ParallelState()
