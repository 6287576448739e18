"""Tensor-parallel serving: one process per GPU, one engine replica per TP group.

Rank 0 of the group owns the C++ scheduler, the HTTP server and the request state; every
rank owns its weight shard, its KV-cache shard (its kv heads) and its hipGraphs.  Each
engine step, rank 0 broadcasts the step header (StepInfo + an eager bit + a launch mode,
10 int64) over a gloo control group -- ONE host broadcast per step: the step inputs
themselves travel as one device broadcast of rank 0's staging region (decode: at the head of
the step, inside the hipGraph, ModelRunner._decode_body -> comm.tp_broadcast, the custom IPC
broadcast kernel when it fits, else RCCL; prefill: ModelRunner._stage_prefill's packed
region).
Decode lookahead works across the group: rank 0 broadcasts a lookahead step's header as it
launches it (mode LAUNCH / CHAINED) and followers replay without waiting on the host
(ModelRunner.replay_decode), so every rank's GPU queue holds the next step.  The
forward's all-reduces (O-proj, down-proj) and the vocab-parallel logits all-gather run on
the custom IPC kernels over xGMI at decode sizes (K13 all-reduce and its all-gather
sibling, parallel/custom_allreduce.py), RCCL above them: a captured decode graph then holds
only our kernels, which is what lets ranks sharing one GPU (gloo control plane) replay it.  Every rank sees the full
logits and runs the same seeded sampler, so all ranks produce identical tokens without
another collective.
"""
from __future__ import annotations

import os
import time
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from ..engine.config import EngineConfig
from ..engine.model_runner import ModelRunner
from ..models.config import get_config
from .state import ParallelState, init_distributed

_INFO_KEYS = ["is_prefill", "num_seqs", "num_tokens", "num_tiles", "num_samples",
              "max_seq_len", "num_preempted", "num_decode", "tile_rows"]
# header = info + eager bit + launch mode.  eager = 1: a decode step rank 0 runs eagerly (a
# request asked for penalties / log-probs) -- every rank then runs that step eagerly too, so
# the group issues one and the same collective sequence (an eager expert-parallel step takes
# the exact-split dispatch, a replayed graph the fixed-capacity one: they must never mix)
EXECUTE, LAUNCH, CHAINED = 0, 1, 2
STOP = -1


def _is_eager_decode(info: dict) -> int:
    return int(not info["is_prefill"] and bool(info.get("extras")))


class TPStepBroadcaster:
    """Wraps rank 0's runner: broadcast the step header, then run the step locally."""

    def __init__(self, runner: ModelRunner, ctrl_group):
        self.runner = runner
        self.ctrl = ctrl_group

    def __getattr__(self, name):
        return getattr(self.runner, name)

    def _header(self, info: dict, mode: int) -> None:
        vals = [int(info.get(k, 0)) for k in _INFO_KEYS]  # (hand-built infos may omit keys)
        head = torch.tensor(vals + [_is_eager_decode(info), mode],
                            dtype=torch.int64)
        dist.broadcast(head, 0, group=self.ctrl)

    def execute(self, info: dict) -> np.ndarray:
        self._header(info, EXECUTE)
        return self.runner.execute(info)

    def launch_decode(self, info: dict, chained: bool = False):
        self._header(info, CHAINED if chained else LAUNCH)
        return self.runner.launch_decode(info, chained=chained)

    def shutdown(self) -> None:
        head = torch.full((len(_INFO_KEYS) + 2,), STOP, dtype=torch.int64)
        dist.broadcast(head, 0, group=self.ctrl)
        dist.barrier(group=self.ctrl)
        dist.destroy_process_group()


def worker_loop(runner: ModelRunner, ctrl_group) -> None:
    """Ranks != 0: mirror every step rank 0 broadcasts until STOP.  Decode steps replay
    without a host wait (their tokens are rank 0's business) unless an expert-parallel
    dispatch may need the step re-run (runner.execute checks the overflow flag)."""
    while True:
        head = torch.zeros(len(_INFO_KEYS) + 2, dtype=torch.int64)
        dist.broadcast(head, 0, group=ctrl_group)
        if int(head[0]) == STOP:
            return
        vals = head.tolist()
        info = {k: int(v) for k, v in zip(_INFO_KEYS, vals)}
        if vals[len(_INFO_KEYS)]:
            runner.execute_decode_eager(info)
        elif not info["is_prefill"] and not runner._ep_moe:
            runner.replay_decode(info)
        else:
            runner.execute(info)


def build_tp(ecfg: EngineConfig, backend: Optional[str] = None, log=print):
    """Initialise the TP group and this rank's runner.  Returns (state, runner, ctrl)."""
    mcfg = get_config(ecfg.model)
    tp = ecfg.tensor_parallel_size
    # IPC staging large enough for the decode step's vocab-parallel logits all-gather
    # (rows x vocab/tp bf16) so every captured decode graph keeps it on the IPC kernel
    rows = max(ecfg.max_num_seqs, ecfg.cuda_graph_max_bs or 0)
    car_bytes = rows * (-(-mcfg.vocab_size // tp) + 64) * 2
    st = init_distributed(tp_size=tp, backend=backend, car_buffer_bytes=car_bytes)
    if st.world_size != ecfg.tensor_parallel_size:
        raise ValueError("one engine replica per job: WORLD_SIZE must equal TP size")
    ctrl = dist.new_group(backend="gloo")
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


def serve_tp(ecfg: EngineConfig, host: str, port: int, telemetry=None) -> None:
    """telemetry(labels) -> text providers of this rank (kernel-stats windows, GPU counters):
    rank 0 serves its own and merges the followers' (written under /dev/shm by a
    rank_metrics.RankMetricsWriter on each follower) into /metrics, rank-labelled."""
    import uvicorn

    from ..exporter import rank_metrics
    from ..server.api_server import build_app

    rank = int(os.environ.get("RANK", "0"))
    tag = f"tp-{os.environ.get('MASTER_PORT', '0')}"
    providers = telemetry({"rank": str(rank)}) if telemetry else []
    writer = None
    if rank != 0 and providers:
        writer = rank_metrics.RankMetricsWriter(tag, rank, providers).start()
    eng, bc = make_tp_engine(ecfg)
    if eng is None:
        if writer is not None:
            writer.stop()
        return
    app, ae = build_app(ecfg, engine=eng)
    ae.telemetry = providers
    ae.rank_metrics_tag = tag
    try:
        uvicorn.run(app, host=host, port=port, log_level="info", access_log=False)
    finally:
        bc.shutdown()
