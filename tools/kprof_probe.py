"""Probe: does an in-process torch.profiler window (started from a side thread, like a metrics
sidecar thread would) see the engine's kernels, including those replayed from hipGraphs?

    python tools/kprof_probe.py
"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams  # noqa: E402
from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine  # noqa: E402


def main():
    eng = LLMEngine(EngineConfig(model="qwen3-0.6b", max_model_len=1024, max_num_seqs=64,
                                 max_num_batched_tokens=4096, device="cuda"))
    stop = threading.Event()

    def serve():
        while not stop.is_set():
            eng.generate(None, SamplingParams(max_tokens=64, temperature=0, ignore_eos=True),
                         prompt_ids=[[10 + i + j for j in range(200)] for i in range(64)])

    th = threading.Thread(target=serve, daemon=True)
    th.start()
    time.sleep(3)
    t0 = time.time()
    p = profile(activities=[ProfilerActivity.CUDA])
    p.start()
    time.sleep(1.0)
    p.stop()
    t1 = time.time()
    stop.set()
    th.join(timeout=60)
    rows = {}
    for e in p.events():
        if e.device_type.name != "CUDA":
            continue
        d = rows.setdefault(e.name, [0, 0.0])
        d[0] += 1
        d[1] += e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total
    tot = sum(v[1] for v in rows.values())
    print(f"window {t1 - t0:.2f}s: {len(rows)} kernels, {tot / 1e3:.1f} ms device time")
    for k, (n, us) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:15]:
        print(f"{us / 1e3:9.2f} ms {n:6d}  {k[:100]}")


if __name__ == "__main__":
    main()
