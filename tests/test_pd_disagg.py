"""Disaggregated prefill/decode across two engine PROCESSES (gloo on CPU here; RCCL over
xGMI on MI355X): the gateway prefills on the prefill server, the decode server pulls
the request's KV blocks with one packed send/recv, and the generated text must equal
a monolithic engine's (same weights, greedy)."""
import asyncio
import os
import socket
import subprocess
import sys
import time
import urllib.request

import aiohttp
import pytest
from aiohttp import web

from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine
from aws_k8s_ansible_provisioner_amd.gateway.picker import PickerConfig
from aws_k8s_ansible_provisioner_amd.gateway.server import Gateway

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--model", "tiny-qwen3", "--device", "cpu", "--max-model-len", "256",
          "--max-num-seqs", "8", "--max-num-batched-tokens", "64", "--block-size", "32",
          "--num-gpu-blocks", "128", "--served-model-name", "Qwen/Qwen3-0.6B"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def pd_servers():
    master = _port()
    procs, urls = [], []
    for rank, role in enumerate(["prefill", "decode"]):
        port = _port()
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(master), AKAP_DIST_BACKEND="gloo",
                   PYTHONPATH=ROOT)
        procs.append(subprocess.Popen(
            [sys.executable, "-m", "aws_k8s_ansible_provisioner_amd.server", *COMMON,
             "--kv-role", role, "--port", str(port), "--host", "127.0.0.1"],
            env=env, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE))
        urls.append(f"http://127.0.0.1:{port}")
    deadline = time.time() + 120
    for u in urls:
        while True:
            try:
                urllib.request.urlopen(u + "/health", timeout=1)
                break
            except Exception:
                if time.time() > deadline or any(p.poll() is not None for p in procs):
                    for p in procs:
                        p.kill()
                    errs = [p.stderr.read().decode()[-2000:] for p in procs]
                    raise RuntimeError(f"P/D servers failed to start: {errs}")
                time.sleep(0.2)
    yield urls
    for p in procs:
        p.kill()
        p.wait()


def test_pd_generation_matches_monolithic(pd_servers):
    pre_url, dec_url = pd_servers
    prompt = "disaggregated prefill and decode over RCCL " * 3
    ref = LLMEngine(EngineConfig(model="tiny-qwen3", device="cpu", max_model_len=256,
                                 max_num_seqs=8, max_num_batched_tokens=64, block_size=32,
                                 num_gpu_blocks=128), log=lambda *a: None)
    expect = ref.generate([prompt], SamplingParams(max_tokens=12, temperature=0,
                                                   ignore_eos=True))[0]

    async def run():
        gw = Gateway([(pre_url, "prefill"), (dec_url, "decode")], [],
                     PickerConfig(pd_threshold_chars=32), scrape_interval=0.2)
        runner = web.AppRunner(gw.app())
        await runner.setup()
        port = _port()
        await web.TCPSite(runner, "127.0.0.1", port).start()
        try:
            await asyncio.sleep(0.3)
            async with aiohttp.ClientSession() as s:
                async with s.post(f"http://127.0.0.1:{port}/v1/completions",
                                  json={"prompt": prompt, "max_tokens": 12, "temperature": 0,
                                        "ignore_eos": True}) as r:
                    assert r.status == 200, await r.text()
                    j = await r.json()
                async with s.post(f"http://127.0.0.1:{port}/v1/completions",
                                  json={"prompt": prompt, "max_tokens": 12, "temperature": 0,
                                        "ignore_eos": True, "stream": True}) as r:
                    sse = await r.text()
            assert gw.m_pd.value() == 2
            return j, sse
        finally:
            await runner.cleanup()

    j, sse = asyncio.run(run())
    assert j["usage"]["completion_tokens"] == 12
    assert j["choices"][0]["text"] == expect.text
    import json as _j
    chunks = [_j.loads(l[6:]) for l in sse.splitlines() if l.startswith("data: {")]
    assert "".join(c["choices"][0]["text"] for c in chunks if c.get("choices")) == \
        "".join(ref.tokenizer.decode_token(t) for t in expect.output_ids)
    # the prefill server released the held blocks after the push
    m = urllib.request.urlopen(pre_url + "/metrics").read().decode()
    assert "vllm:gpu_cache_usage_perc" in m


_PD_WORKER = r"""
import json, os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine
from aws_k8s_ansible_provisioner_amd.parallel.pd_driver import PDPair
rank = int(os.environ["RANK"])
dist.init_process_group("gloo", rank=rank, world_size=2)
eng = LLMEngine(EngineConfig(model="tiny-qwen3", device="cpu", max_model_len=256, max_num_seqs=8,
                             max_num_batched_tokens=64, block_size=32, num_gpu_blocks=128,
                             kv_role="prefill" if rank == 0 else "decode"), log=lambda *a: None)
pair = PDPair(eng, rank, 2, ctrl_group=dist.new_group(backend="gloo"))
prompts = [list(range(5, 5 + 30 + 7 * i)) for i in range(5)]
sp = SamplingParams(max_tokens=9, temperature=0, ignore_eos=True)
outs = {}
if rank == 0:
    pair.run_prefill(prompts, sp)
else:
    orig = eng.step
    def step():
        res = orig()
        for o in res:
            if o.finished:
                outs[len(o.prompt_ids)] = o.output_ids
        return res
    eng.step = step
    r = pair.run_decode(sp)
    assert r["finished"] == 5 and r["output_tokens"] == 45, r
    print("PD_OUT " + json.dumps({str(k): v for k, v in outs.items()}), flush=True)
pair.close()
dist.barrier()
dist.destroy_process_group()
"""


def test_pd_driver_matches_monolithic(tmp_path):
    """bench.py --mode pd's in-process P/D data path (gloo, 2 ranks) == monolithic greedy."""
    import json
    import os
    import socket
    import subprocess
    import sys

    script = tmp_path / "pd_worker.py"
    script.write_text(_PD_WORKER)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), REPO=repo)
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e.decode()[-3000:]
    line = [ln for ln in outs[1][0].decode().splitlines() if ln.startswith("PD_OUT ")][0]
    got = json.loads(line[len("PD_OUT "):])
    ref = LLMEngine(EngineConfig(model="tiny-qwen3", device="cpu", max_model_len=256,
                                 max_num_seqs=8, max_num_batched_tokens=64, block_size=32,
                                 num_gpu_blocks=128), log=lambda *a: None)
    prompts = [list(range(5, 5 + 30 + 7 * i)) for i in range(5)]
    exp = ref.generate(None, SamplingParams(max_tokens=9, temperature=0, ignore_eos=True),
                       prompt_ids=prompts)
    for p_, o in zip(prompts, exp):
        assert got[str(len(p_))] == o.output_ids
