"""Tensor-parallel serving: one process per GPU, one engine replica per TP group.

Rank 0 of the group owns the C++ scheduler, the HTTP server and the request state; every
rank owns its weight shard, its KV-cache shard (its kv heads) and its hipGraphs.  Each
engine step, rank 0 broadcasts the step header (StepInfo, 9 int64) over a gloo control
group -- ONE host broadcast per decode step: the decode inputs themselves travel as one
RCCL broadcast of rank 0's device staging region at the head of the decode step (inside the
hipGraph, ModelRunner._decode_body).  Prefill steps also send the used prefix of the pinned
batch buffers (~KBs) as a second gloo broadcast, sized by the header.  The
forward's all-reduces (O-proj, down-proj) and the vocab-parallel logits all-gather run on
RCCL over xGMI (and are captured inside the decode hipGraphs).  Every rank sees the full
logits and runs the same seeded sampler, so all ranks produce identical tokens without
another collective.
"""
from __future__ import annotations

import time
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from ..engine.config import EngineConfig
from ..engine.model_runner import ModelRunner
from ..models.config import get_config
from .state import ParallelState, init_distributed

_STEP_KEYS = ["input_ids", "positions", "slots", "seq_lens", "q_start", "block_tables",
              "tile_seq", "tile_row", "logits_idx", "temperature", "top_p", "top_k", "seeds",
              "steps"]
_INFO_KEYS = ["is_prefill", "num_seqs", "num_tokens", "num_tiles", "num_samples",
              "max_seq_len", "num_preempted", "num_decode"]
# header = info + payload bytes (0 for decode steps: inputs go by the in-graph broadcast)
STOP = -1


def _extent(key: str, info: dict, runner: ModelRunner) -> int:
    B, T, S = info["num_seqs"], info["num_tokens"], info["num_samples"]
    if not info["is_prefill"]:
        B = T = S = max(B, 1)
        for b in runner.buckets:  # decode replays pad rows up to the bucket
            if b >= info["num_seqs"]:
                B = T = S = b
                break
    return {"input_ids": T, "positions": T, "slots": T, "seq_lens": B, "q_start": B + 1,
            "block_tables": B * runner.max_blocks, "tile_seq": info["num_tiles"],
            "tile_row": info["num_tiles"], "logits_idx": S, "temperature": S, "top_p": S,
            "top_k": S, "seeds": S, "steps": S}[key]


class TPStepBroadcaster:
    """Wraps rank 0's runner: broadcast the step, then execute it locally."""

    def __init__(self, runner: ModelRunner, ctrl_group):
        self.runner = runner
        self.ctrl = ctrl_group

    def __getattr__(self, name):
        return getattr(self.runner, name)

    def execute(self, info: dict) -> np.ndarray:
        r = self.runner
        payload = None
        if info["is_prefill"]:
            parts = [torch.from_numpy(r.np[k][:_extent(k, info, r)].view(np.uint8).copy())
                     for k in _STEP_KEYS]
            payload = torch.cat(parts)
        head = torch.tensor([info[k] for k in _INFO_KEYS] +
                            [0 if payload is None else payload.numel()], dtype=torch.int64)
        dist.broadcast(head, 0, group=self.ctrl)
        if payload is not None:
            dist.broadcast(payload, 0, group=self.ctrl)
        return r.execute(info)

    def shutdown(self) -> None:
        head = torch.full((len(_INFO_KEYS) + 1,), STOP, dtype=torch.int64)
        dist.broadcast(head, 0, group=self.ctrl)
        dist.barrier(group=self.ctrl)
        dist.destroy_process_group()


def worker_loop(runner: ModelRunner, ctrl_group) -> None:
    """Ranks != 0: mirror every step rank 0 broadcasts until STOP."""
    while True:
        head = torch.zeros(len(_INFO_KEYS) + 1, dtype=torch.int64)
        dist.broadcast(head, 0, group=ctrl_group)
        if int(head[0]) == STOP:
            return
        vals = head.tolist()
        info = {k: int(v) for k, v in zip(_INFO_KEYS, vals)}
        if vals[-1]:
            payload = torch.empty(int(vals[-1]), dtype=torch.uint8)
            dist.broadcast(payload, 0, group=ctrl_group)
            off = 0
            for k in _STEP_KEYS:
                cnt = _extent(k, info, runner)
                arr = runner.np[k]
                nbytes = cnt * arr.itemsize
                arr[:cnt] = payload[off:off + nbytes].numpy().view(arr.dtype)
                off += nbytes
        runner.execute(info)


def build_tp(ecfg: EngineConfig, backend: Optional[str] = None, log=print):
    """Initialise the TP group and this rank's runner.  Returns (state, runner, ctrl)."""
    st = init_distributed(tp_size=ecfg.tensor_parallel_size, backend=backend)
    if st.world_size != ecfg.tensor_parallel_size:
        raise ValueError("one engine replica per job: WORLD_SIZE must equal TP size")
    ctrl = dist.new_group(backend="gloo")
    mcfg = get_config(ecfg.model)
    runner = ModelRunner(ecfg, mcfg, st, log=log if st.rank == 0 else (lambda *a: None))
    return st, runner, ctrl


def make_tp_engine(ecfg: EngineConfig, backend: Optional[str] = None, log=print):
    """Rank 0 -> (LLMEngine, broadcaster); other ranks block in worker_loop and
    return (None, None) when rank 0 shuts down."""
    from ..engine.llm_engine import LLMEngine

    st, runner, ctrl = build_tp(ecfg, backend, log)
    if st.rank != 0:
        worker_loop(runner, ctrl)
        dist.barrier(group=ctrl)
        dist.destroy_process_group()
        return None, None
    bc = TPStepBroadcaster(runner, ctrl)
    eng = LLMEngine(ecfg, runner.mcfg, st, log=log, runner=bc)
    return eng, bc


def serve_tp(ecfg: EngineConfig, host: str, port: int) -> None:
    import uvicorn

    from ..server.api_server import build_app

    eng, bc = make_tp_engine(ecfg)
    if eng is None:
        return
    app, ae = build_app(ecfg, engine=eng)
    try:
        uvicorn.run(app, host=host, port=port, log_level="info", access_log=False)
    finally:
        bc.shutdown()
