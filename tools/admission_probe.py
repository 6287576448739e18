#!/usr/bin/env python3
"""Host timeline of a headline-bench wave's opening (round 6): where the time between
`generate()` and the first prefill kernel goes, and when each prefill step's tokens reach the
host.  Same engine config and workload as `bench.py` (Qwen3-0.6B, 256 x 512-token prompts,
16,384-token steps); one warmup wave, then one instrumented wave.

    python tools/admission_probe.py [--lists]   (--lists: prompts as Python lists)
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams  # noqa
from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lists", action="store_true")
    ap.add_argument("--output-len", type=int, default=256)
    a = ap.parse_args()
    import torch

    eng = LLMEngine(EngineConfig(model="qwen3-0.6b", max_model_len=2048, max_num_seqs=256,
                                 max_num_batched_tokens=16384, block_size=32, device="cuda",
                                 gpu_memory_utilization=0.9), log=lambda *x: None)
    sp = SamplingParams(max_tokens=a.output_len, temperature=0.0, ignore_eos=True)
    rng = np.random.default_rng(7)

    def prompts():
        p = rng.integers(10, 150000, size=(256, 512), dtype=np.int32)
        return [r.tolist() for r in p] if a.lists else p

    eng.generate(None, sp, prompt_ids=prompts())  # warmup wave
    torch.cuda.synchronize()
    marks = []
    r = eng.runner
    orig_exec, orig_fwd, orig_step = r.execute_prefill, r.model.forward, eng.step

    def exec_prefill(info):
        marks.append(("execute_prefill entered", time.perf_counter()))
        return orig_exec(info)

    def fwd(*x, **k):
        marks.append(("forward entered", time.perf_counter()))
        return orig_fwd(*x, **k)

    def step():
        out = orig_step()
        if len([m for m in marks if m[0].startswith("step")]) < 10:
            marks.append((f"step returned ({len(out)} outputs)", time.perf_counter()))
        return out

    r.execute_prefill, r.model.forward, eng.step = exec_prefill, fwd, step
    P = prompts()
    t0 = time.perf_counter()
    names = []
    params = sp.normalized()
    for p in P:
        names.append(eng._add(None, None, params, p))
    t_add = time.perf_counter()
    arrivals = sorted(st.arrival for st in eng.reqs.values())
    outs = {}
    while eng.has_unfinished():
        for o in eng.step():
            if o.finished:
                outs[o.req_id] = o
    t_end = time.perf_counter()
    ttft = sorted(o.ttft for o in outs.values() if o.ttft is not None)
    print(f"adds: 256 requests in {1e3 * (t_add - t0):.2f} ms "
          f"(arrival spread {1e3 * (arrivals[-1] - arrivals[0]):.2f} ms)")
    for name, t in marks[:30]:
        print(f"  +{1e3 * (t - t0):8.2f} ms  {name}")
    print(f"wave {1e3 * (t_end - t0):.1f} ms, p50 TTFT {1e3 * ttft[len(ttft) // 2]:.2f} ms, "
          f"min {1e3 * ttft[0]:.2f}, max {1e3 * ttft[-1]:.2f}")
    print("timers:", {k: round(v, 4) for k, v in eng.timers.items()})
    return 0


if __name__ == "__main__":
    sys.exit(main())
