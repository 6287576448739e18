"""Tensor parallelism across 2 processes (gloo on CPU; RCCL over xGMI on MI355X):
vocab-parallel embedding/LM head, head-split attention with its own KV-cache shard,
row/column-split MLP with all-reduce, rank-0 scheduling with step broadcast.  Outputs
must match the single-process model with the same logical weights."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
import torch
sys.path.insert(0, os.environ["ROOT"])
from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
from aws_k8s_ansible_provisioner_amd.parallel.tp_worker import make_tp_engine
model = os.environ["MODEL"]
ecfg = EngineConfig(model=model, device="cpu", max_model_len=256, max_num_seqs=8,
                    max_num_batched_tokens=32, block_size=32, num_gpu_blocks=96,
                    tensor_parallel_size=int(os.environ["WORLD_SIZE"]), shard_init="full",
                    init_std=0.15)
eng, bc = make_tp_engine(ecfg, backend="gloo", log=lambda *a: None)
if eng is not None:
    outs = eng.generate(None, SamplingParams(max_tokens=8, temperature=0, ignore_eos=True),
                        prompt_ids=[list(range(5, 40)), [100, 101], [9, 9, 9]])
    bc.shutdown()
    print("RESULT " + json.dumps([o.output_ids for o in outs]), flush=True)
from aws_k8s_ansible_provisioner_amd.models.moe import MoEBlock
print("FALLBACKS", MoEBlock.ep_fallbacks, MoEBlock.ep_exact_layers, flush=True)
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("model,moe_mode,world,ep_fixed", [
    ("tiny-llama", "tp", 2, 512), ("tiny-qwen3", "tp", 2, 512), ("tiny-mixtral", "tp", 2, 512),
    ("tiny-mixtral", "ep", 2, 512),
    # 4 ranks: kv heads replicated (2 kv heads / 4 ranks), one expert per EP rank; EP with the
    # fixed-capacity (graph-safe) dispatch and with the exact-split prefill path
    ("tiny-llama", "tp", 4, 512), ("tiny-mixtral", "ep", 4, 512), ("tiny-mixtral", "ep", 4, 0),
    # the real world-8 layouts: Llama-3-70B's one KV head per TP rank (GQA 8 -> 2 q heads and
    # 1 kv head per rank) and Mixtral's one expert per EP rank, fixed-capacity dispatch (slack
    # 2) and the exact path; slack 0.3 forces dispatch overflows -> every layer falls back
    ("tiny-llama-kv8", "tp", 8, 512), ("tiny-mixtral8", "ep", 8, 512),
    ("tiny-mixtral8", "ep", 8, 0), ("tiny-mixtral8", "ep-slack0.3", 8, 512)])
def test_tp_matches_tp1(model, moe_mode, world, ep_fixed):
    from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
    from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine

    port = _port()
    procs = []
    for r in range(world):
        mode, _, slack = moe_mode.partition("-slack")
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ROOT=ROOT, MODEL=model,
                   AKAP_MOE_MODE=mode, AKAP_EP_FIXED_MAX_T=str(ep_fixed),
                   AKAP_EP_SLACK=slack or "2.0", AKAP_EP_MIN_CAP="1" if slack else "8",
                   OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, "-c", CHILD], env=env, cwd=ROOT,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-3000:] for o in outs]
    line = [l for l in outs[0][0].splitlines() if l.startswith("RESULT ")][0]
    tp_out = json.loads(line[7:])
    fb = [l for l in outs[0][0].splitlines() if l.startswith("FALLBACKS ")][0].split()
    if "slack" in moe_mode:  # the undersized dispatch overflowed: steps re-ran exactly
        assert int(fb[1]) > 0, fb
    elif moe_mode == "ep" and ep_fixed:
        # prefill and decode steps alike on the fixed dispatch: no step re-run, no layer on
        # the host-synced exact path
        assert int(fb[1]) == 0 and int(fb[2]) == 0, fb
    ref = LLMEngine(EngineConfig(model=model, device="cpu", max_model_len=256, max_num_seqs=8,
                                 max_num_batched_tokens=32, block_size=32, num_gpu_blocks=96,
                                 shard_init="full", init_std=0.15), log=lambda *a: None)
    from aws_k8s_ansible_provisioner_amd.models.reference_forward import dense_logits

    prompts = [list(range(5, 40)), [100, 101], [9, 9, 9]]
    # identical logical weights: every TP token must be (near-)argmax of the dense fp32
    # reference (bf16 partial sums reduced across ranks may flip exact near-ties)
    for p, out in zip(prompts, tp_out):
        logits = dense_logits(ref.runner.model, p + out).float()
        for i, tok in enumerate(out):
            row = logits[len(p) - 1 + i]
            gap = (row.max() - row[tok]).item() / (row.std().item() + 1e-6)
            assert gap <= 0.1, (i, tok, gap)


FUSED_CHILD = r"""
import json, os, sys
import torch
sys.path.insert(0, os.environ["ROOT"]); sys.path.insert(0, os.path.join(os.environ["ROOT"], "tests"))
from aws_k8s_ansible_provisioner_amd.parallel.state import init_distributed
from aws_k8s_ansible_provisioner_amd.models.config import get_config
from aws_k8s_ansible_provisioner_amd.models.transformer import DecoderLM
from test_fused_decode import PLAIN_PLAN
import test_fused_decode as tfd
ps = init_distributed(tp_size=int(os.environ["WORLD_SIZE"]), backend="gloo")
m, batch, ids, ks, vs = tfd._setup(os.environ["MODEL"], "cpu")
# _setup builds an unsharded model: rebuild the TP shard with the same logical weights
cfg = get_config(os.environ["MODEL"])
m = DecoderLM(cfg, device="cpu", seed=0, max_model_len=256, init_std=0.05, pstate=ps,
              full_then_shard=True)
kv = m.allocate_kv_cache(ks[0].shape[0], 32)
torch.manual_seed(1)
kv.copy_((torch.randn(kv.shape) * 0.5).to(kv.dtype))
ks, vs = m.cache_views(kv, 32)
base = m.forward(ids, batch, ks, vs).float()
fused = m._forward_fused_decode(ids, batch, ks, vs, PLAIN_PLAN).float()
if ps.rank == 0:
    print("RESULT " + json.dumps({"err": (fused - base).abs().max().item(),
                                  "scale": base.abs().max().item()}), flush=True)
# orderly teardown: a rank that exits while its peer still has gloo work queued can die in
# std::terminate from the process group's threads
import torch.distributed as dist
dist.barrier()
dist.destroy_process_group()
"""


@pytest.mark.parametrize("model", ["tiny-qwen3", "tiny-llama"])
def test_tp2_fused_decode_chain_matches_unfused(model):
    """The fused decode chain at tp=2: row-parallel O / down partial sums reach the residual
    epilogue through comm.tp_all_reduce_resnorm (RCCL + epilogue here; the custom xGMI kernel
    with the epilogue fused on MI355X) and equal the unfused TP forward."""
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ROOT=ROOT, MODEL=model)
        procs.append(subprocess.Popen([sys.executable, "-c", FUSED_CHILD], env=env, cwd=ROOT,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-3000:] for o in outs]
    res = json.loads([l for l in outs[0][0].splitlines() if l.startswith("RESULT ")][0][7:])
    assert res["err"] <= 3e-2 * res["scale"] + 3e-2, res


def test_tp_step_is_one_host_broadcast(monkeypatch):
    """Rank 0 sends every step to the other TP ranks with ONE gloo broadcast (the header): the
    inputs go by RCCL broadcasts of rank 0's device staging regions (the decode graph's first
    op; ModelRunner._stage_prefill for prefill steps).  Lookahead launches carry their mode."""
    import torch.distributed as dist

    from aws_k8s_ansible_provisioner_amd.parallel import tp_worker

    sent = []
    monkeypatch.setattr(dist, "broadcast", lambda t, src, group=None: sent.append(t.clone()))

    class FakeRunner:
        buckets = [1, 2, 4]

        def execute(self, info):
            return "ran"

        def launch_decode(self, info, chained=False):
            return ("launched", chained)

    bc = tp_worker.TPStepBroadcaster(FakeRunner(), ctrl_group=None)
    dec = {"is_prefill": 0, "num_seqs": 3, "num_tokens": 3, "num_tiles": 0,
           "num_samples": 3, "max_seq_len": 9, "num_preempted": 0, "num_decode": 3,
           "tile_rows": 0}
    assert bc.execute(dec) == "ran"
    assert len(sent) == 1 and sent[0].tolist()[-1] == tp_worker.EXECUTE
    assert sent[0].tolist()[-2] == 0  # graph-replayable decode step
    sent.clear()
    # a decode step with extras (log-probs / penalties) runs eagerly on rank 0: the header's
    # eager bit makes every follower run it eagerly as well
    bc.execute(dict(dec, extras={"logprobs": True}))
    assert len(sent) == 1 and sent[0].tolist()[-2] == 1
    sent.clear()
    pre = dict(dec, is_prefill=1, num_tokens=20, num_tiles=2, num_decode=0)
    bc.execute(pre)
    assert len(sent) == 1 and sent[0].tolist()[0] == 1
    sent.clear()
    assert bc.launch_decode(dec, chained=True) == ("launched", True)
    assert len(sent) == 1 and sent[0].tolist()[-1] == tp_worker.CHAINED


def test_tp_follower_mirrors_eager_decode(monkeypatch):
    """under TP x EP a decode step rank 0 runs eagerly must not meet a
    follower's graph replay (eager EP = exact-split all_to_alls, graph = fixed-capacity ones:
    the collective sequences differ).  The follower loop routes eager-bit headers to
    ModelRunner.execute_decode_eager and everything else as before."""
    import torch
    import torch.distributed as dist

    from aws_k8s_ansible_provisioner_amd.parallel import tp_worker

    dec = {"is_prefill": 0, "num_seqs": 3, "num_tokens": 3, "num_tiles": 0,
           "num_samples": 3, "max_seq_len": 9, "num_preempted": 0, "num_decode": 3,
           "tile_rows": 0}
    heads = [[dec[k] for k in tp_worker._INFO_KEYS] + [1, tp_worker.EXECUTE],
             [dec[k] for k in tp_worker._INFO_KEYS] + [0, tp_worker.EXECUTE],
             [tp_worker.STOP] * (len(tp_worker._INFO_KEYS) + 2)]

    def fake_bcast(t, src, group=None):
        t.copy_(torch.tensor(heads.pop(0), dtype=torch.int64))

    monkeypatch.setattr(dist, "broadcast", fake_bcast)
    calls = []

    class Follower:
        _ep_moe = True

        def execute_decode_eager(self, info):
            calls.append(("eager", info["num_seqs"]))

        def execute(self, info):
            calls.append(("execute", info["num_seqs"]))

        def replay_decode(self, info):
            calls.append(("replay", info["num_seqs"]))

    tp_worker.worker_loop(Follower(), ctrl_group=None)
    assert calls == [("eager", 3), ("execute", 3)]


EP_EXTRAS_CHILD = r"""
import json, os, sys
sys.path.insert(0, os.environ["ROOT"])
from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
from aws_k8s_ansible_provisioner_amd.parallel.tp_worker import make_tp_engine
ecfg = EngineConfig(model="tiny-mixtral", device="cpu", max_model_len=256, max_num_seqs=8,
                    max_num_batched_tokens=32, block_size=32, num_gpu_blocks=96,
                    tensor_parallel_size=2, shard_init="full", init_std=0.15)
eng, bc = make_tp_engine(ecfg, backend="gloo", log=lambda *a: None)
if eng is not None:
    ps = [SamplingParams(max_tokens=6, temperature=0, ignore_eos=True, logprobs=1),
          SamplingParams(max_tokens=6, temperature=0, ignore_eos=True,
                         repetition_penalty=1.0, presence_penalty=0.5)]
    names = [eng.add_request(None, None, p, prompt_ids=q)
             for q, p in zip([list(range(5, 30)), [7, 8, 9]], ps)]
    final = {}
    while eng.has_unfinished():
        for o in eng.step():
            if o.finished:
                final[o.req_id] = o.output_ids
    bc.shutdown()
    print("RESULT " + json.dumps([final[n] for n in names]), flush=True)
"""


def test_tp_ep_decode_with_logprobs_and_penalties():
    """TP x EP (tiny-Mixtral, 2 ranks, exact-split eager dispatch) with a log-probs request and
    a penalty request in the batch: every step carries extras, the followers mirror the eager
    steps and the group finishes (no collective mismatch / hang)."""
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ROOT=ROOT,
                   AKAP_MOE_MODE="ep", AKAP_EP_FIXED_MAX_T="0", OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, "-c", EP_EXTRAS_CHILD], env=env, cwd=ROOT,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-3000:] for o in outs]
    line = [l for l in outs[0][0].splitlines() if l.startswith("RESULT ")][0]
    res = json.loads(line[7:])
    assert [len(r) for r in res] == [6, 6]


LOOKAHEAD_CHILD = r"""
import json, os, sys
sys.path.insert(0, os.environ["ROOT"])
from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
from aws_k8s_ansible_provisioner_amd.parallel.tp_worker import make_tp_engine
ecfg = EngineConfig(model="tiny-llama", device="cpu", max_model_len=256, max_num_seqs=8,
                    max_num_batched_tokens=64, block_size=32, num_gpu_blocks=96,
                    tensor_parallel_size=2, shard_init="full", init_std=0.15)
eng, bc = make_tp_engine(ecfg, backend="gloo", log=lambda *a: None)
if eng is not None:
    prompts = [list(range(5, 40)), [100, 101], [9, 9, 9], list(range(300, 310))]
    params = [SamplingParams(max_tokens=m, temperature=0, ignore_eos=True) for m in (5, 9, 14)]
    params.append(SamplingParams(max_tokens=12, temperature=0.8, top_p=0.9, seed=3,
                                 ignore_eos=True))
    names = [eng.add_request(None, None, p, prompt_ids=q) for q, p in zip(prompts, params)]
    final = {}
    while eng.has_unfinished():
        for o in eng.step():
            if o.finished:
                final[o.req_id] = o.output_ids
    bc.shutdown()
    print("RESULT " + json.dumps({"out": [final[n] for n in names],
                                  "lookahead": eng.lookahead_steps}), flush=True)
"""


def test_tp2_lookahead_matches_synchronous():
    """Decode lookahead on a TP group (gloo): rank 0 broadcasts each lookahead step's header
    as it launches it, followers replay it; the token streams equal the synchronous loop's."""
    res = {}
    for mode in ("0", "force"):
        port = _port()
        procs = []
        for r in range(2):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ROOT=ROOT,
                       AKAP_ASYNC_DECODE=mode, OMP_NUM_THREADS="2")
            procs.append(subprocess.Popen([sys.executable, "-c", LOOKAHEAD_CHILD], env=env,
                                          cwd=ROOT, stdout=subprocess.PIPE,
                                          stderr=subprocess.PIPE, text=True))
        outs = [p.communicate(timeout=300) for p in procs]
        assert all(p.returncode == 0 for p in procs), [o[1][-3000:] for o in outs]
        line = [l for l in outs[0][0].splitlines() if l.startswith("RESULT ")][0]
        res[mode] = json.loads(line[7:])
    assert res["0"]["lookahead"] == 0 and res["force"]["lookahead"] > 0, res
    assert res["force"]["out"] == res["0"]["out"]


AGREE_CHILD = r"""
import os, sys
sys.path.insert(0, os.environ["ROOT"])
from aws_k8s_ansible_provisioner_amd.parallel.state import init_distributed
from aws_k8s_ansible_provisioner_amd.parallel import comm
import torch.distributed as dist
ps = init_distributed(tp_size=2, backend="gloo")
# rank 1's tuning-cache file is missing: every rank must take the retune branch
mine = ps.rank != 1
print("RESULT", int(comm.tp_all_true(mine)), int(comm.tp_all_true(True)), flush=True)
dist.barrier()
dist.destroy_process_group()
"""


def test_tp_ranks_agree_on_tuning_cache_load():
    """a rank whose GEMM tuning-cache file is missing/stale retunes (tune_fused then
    broadcasts over the TP group) -- every rank must take that branch, so the load decision is
    a MIN all-reduce over the TP group (model_runner.capture_graphs -> comm.tp_all_true)."""
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ROOT=ROOT)
        procs.append(subprocess.Popen([sys.executable, "-c", AGREE_CHILD], env=env, cwd=ROOT,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-3000:] for o in outs]
    for o in outs:
        line = [l for l in o[0].splitlines() if l.startswith("RESULT")][0]
        assert line.split()[1:] == ["0", "1"], line


def test_ep_dispatch_bytes_bounded():
    """The fixed-capacity EP dispatch moves at most 2x the exact T*K*d rows per all-to-all at
    decode sizes (a per-peer capacity of T*K moved ep x the exact traffic)."""
    import torch

    from aws_k8s_ansible_provisioner_amd.models.config import get_config
    from aws_k8s_ansible_provisioner_amd.models.moe import MoEBlock
    from aws_k8s_ansible_provisioner_amd.parallel.state import ParallelState

    cfg = get_config("tiny-mixtral8")
    for ep in (2, 4, 8):
        ps = ParallelState(rank=0, world_size=ep, tp_size=ep)
        blk = MoEBlock(cfg, ps, "cpu", torch.bfloat16, torch.Generator().manual_seed(0),
                       full_then_shard=False, mode="ep")
        for T in (64, 128, 256, 512):
            exact = T * cfg.experts_per_token
            assert blk.a2a_rows(T) <= 2 * exact, (ep, T, blk.a2a_rows(T), exact)
        # one-token steps: capacity covers every pair (no overflow possible)
        assert blk.ep_capacity(cfg.experts_per_token) == cfg.experts_per_token


def test_car_grid_agreed_from_physical_devices():
    """the K13 grid is one value for the whole communicator -- the minimum of the
    ranks' overrides and of the sharing rule, where sharing is counted from gathered physical
    device keys (one visible GPU per rank is NOT sharing)."""
    from aws_k8s_ansible_provisioner_amd.parallel.custom_allreduce import agree_grid

    own = ["h:0:1:0", "h:0:2:0", "h:0:3:0", "h:0:4:0"]
    assert agree_grid(own, [128] * 4) == 128            # 4 GPUs, index 0 visible in each rank
    assert agree_grid(["h:0:1:0"] * 4, [128] * 4) == 32  # 4 ranks on one GPU
    assert agree_grid(["h:0:1:0"] * 2 + ["h:0:2:0"] * 2, [128] * 4) == 64
    assert agree_grid(own, [128, 128, 16, 128]) == 16   # one rank's override binds everyone
