"""Disaggregated prefill/decode on the GPU, end to end: a prefill server and a decode server
(two processes sharing ONE MI355X), the gateway in front pairing them.  Both KV transports:
  ipc  the decode engine maps the prefill engine's cache (hipIpc) and pulls the request's
       blocks + fills its V tail with one kv_pull launch (/kv/lease ... /kv/done);
  p2p  /kv/push -> packed send over a host-staged gloo channel -> unpack, activate() fills
       the V tail.
A completion through the gateway takes the P/D path and must produce exactly the monolithic
engine's tokens on the same weights."""
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

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--model", "tiny-qwen3", "--device", "cuda", "--max-model-len", "256",
          "--max-num-seqs", "8", "--max-num-batched-tokens", "64", "--block-size", "32",
          "--num-gpu-blocks", "128", "--served-model-name", "Qwen/Qwen3-0.6B"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("bootstrap", ["launcher", "http"])
@pytest.mark.parametrize("transport", ["ipc", "p2p"])
def test_pd_through_the_gateway_on_gpu_matches_monolithic(transport, bootstrap):
    """bootstrap "launcher": both servers are ranks of one torch.distributed job (one pod);
    "http": two INDEPENDENTLY started server processes (the two-pod form: no RANK /
    WORLD_SIZE / MASTER_ADDR) whose KV channel the decode server forms on first use over HTTP
    (p2p: a gloo pair group -- RCCL places no two ranks on one GPU)."""
    from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
    from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine
    from aws_k8s_ansible_provisioner_amd.gateway.picker import PickerConfig
    from aws_k8s_ansible_provisioner_amd.gateway.server import Gateway

    master = _port()
    procs, urls = [], []
    try:
        for rank, role in enumerate(["prefill", "decode"]):
            port = _port()
            extra = []
            if bootstrap == "launcher":
                env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank),
                           MASTER_ADDR="127.0.0.1", MASTER_PORT=str(master),
                           AKAP_DIST_BACKEND="gloo", PYTHONPATH=ROOT, AKAP_KV_TRANSPORT=transport)
            else:
                env = {k: v for k, v in os.environ.items() if k not in
                       ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
                env.update(PYTHONPATH=ROOT, AKAP_KV_TRANSPORT=transport, AKAP_PD_GROUP="pd2",
                           AKAP_PD_PAIR_BACKEND="gloo")
                extra = ["--pd-bootstrap", "http", "--kv-store-port", str(_port())]
            procs.append(subprocess.Popen(
                [sys.executable, "-m", "aws_k8s_ansible_provisioner_amd.server", *COMMON,
                 "--kv-role", role, "--port", str(port), "--host", "127.0.0.1", *extra],
                env=env, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE))
            urls.append(f"http://127.0.0.1:{port}")
        deadline = time.time() + 240
        for u in urls:
            while True:
                try:
                    urllib.request.urlopen(u + "/health", timeout=1)
                    break
                except Exception:
                    if time.time() > deadline or any(p.poll() is not None for p in procs):
                        errs = [p.stderr.read().decode()[-2000:] if p.poll() is not None else ""
                                for p in procs]
                        raise RuntimeError(f"P/D servers failed to start: {errs}")
                    time.sleep(0.5)
        prompt = "disaggregated prefill and decode on one MI355X " * 3

        async def run():
            g = "pd2" if bootstrap == "http" else ""
            gw = Gateway([(urls[0], "prefill", g), (urls[1], "decode", g)], [],
                         PickerConfig(pd_threshold_chars=32), scrape_interval=0.2)
            runner = web.AppRunner(gw.app())
            await runner.setup()
            port = _port()
            await web.TCPSite(runner, "127.0.0.1", port).start()
            try:
                await asyncio.sleep(0.5)
                async with aiohttp.ClientSession() as s:
                    async with s.post(f"http://127.0.0.1:{port}/v1/completions",
                                      json={"prompt": prompt, "max_tokens": 12,
                                            "temperature": 0, "ignore_eos": True}) as r:
                        assert r.status == 200, await r.text()
                        j = await r.json()
                return j, gw.m_pd.value()
            finally:
                await runner.cleanup()

        j, n_pd = asyncio.run(run())
        assert n_pd == 1 and j["usage"]["completion_tokens"] == 12
        ref = LLMEngine(EngineConfig(model="tiny-qwen3", device="cuda", max_model_len=256,
                                     max_num_seqs=8, max_num_batched_tokens=64, block_size=32,
                                     num_gpu_blocks=128), log=lambda *a: None)
        expect = ref.generate([prompt], SamplingParams(max_tokens=12, temperature=0,
                                                       ignore_eos=True))[0]
        assert j["choices"][0]["text"] == expect.text
    finally:
        for p in procs:
            p.kill()
            p.wait()
