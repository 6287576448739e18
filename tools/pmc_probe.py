"""GPU probe of the in-process counter tool (libakap_pmc.so + exporter/pmc_sampler.py).

Run with the tool loaded at process start:
    ROCP_TOOL_LIBRARIES=$PWD/aws_k8s_ansible_provisioner_amd/libakap_pmc.so python tools/pmc_probe.py
Reads the device counters around known work -- a streaming read of a 4 GiB tensor (bytes
known) and a large bf16 matmul (MFMA busy) -- and prints the sampler's rates and its
/metrics text, so the counter semantics (cumulative vs per-read) and the byte calibration are
checked against work whose size is known."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aws_k8s_ansible_provisioner_amd.exporter.pmc_sampler import PMCSampler  # noqa: E402


def main() -> int:
    torch.cuda.init()
    x = torch.ones(1 << 30, dtype=torch.float32, device="cuda")  # 4 GiB
    torch.cuda.synchronize()
    s = PMCSampler(interval_s=1.0, labels={"rank": "0"})
    print("tool status:", s.status(), flush=True)
    ok = s.once()
    print("first read ok:", ok, "names:", s.names, "cumulative:", s.cumulative,
          "error:", s.last_error, flush=True)
    res = {"status": s.status(), "names": s.names, "cumulative": s.cumulative}
    # streaming read: 20 passes over 4 GiB = 85.9 GB
    t0 = time.time()
    for _ in range(20):
        x.sum()
    torch.cuda.synchronize()
    dt = time.time() - t0
    s.once()
    rd = s.derived().get("mem_read_bytes_per_second", 0.0)
    # the read interval spans the 20 passes (plus a few ms of host time around them)
    res["stream"] = {"known_read_bytes_per_second": 20 * 4 * 2**30 / dt, "seconds": dt,
                     "counted_read_bytes_per_second": rd, "rates": s.rates}
    print("stream rates:", json.dumps(s.rates), flush=True)
    # MFMA: 8192^3 bf16 matmuls
    a = torch.randn(8192, 8192, dtype=torch.bfloat16, device="cuda")
    b = torch.randn(8192, 8192, dtype=torch.bfloat16, device="cuda")
    c = torch.empty_like(a)
    for _ in range(3):
        torch.matmul(a, b, out=c)
    torch.cuda.synchronize()
    s.once()
    t0 = time.time()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 0
    while time.time() - t0 < 1.5:  # ~1.5 s of back-to-back MFMA-bound work
        for _ in range(20):
            torch.matmul(a, b, out=c)
        n += 20
        torch.cuda.synchronize()
    e1.record()
    torch.cuda.synchronize()
    gpu_s = e0.elapsed_time(e1) / 1e3
    s.once()
    res["matmul"] = {"derived": s.derived(), "rates": s.rates, "gpu_seconds": gpu_s,
                     "host_seconds": time.time() - t0,
                     "tflops": n * 2 * 8192 ** 3 / gpu_s / 1e12}
    print("matmul derived:", json.dumps(s.derived()), "tflops", res["matmul"]["tflops"],
          "rates", json.dumps(s.rates), flush=True)
    # idle
    time.sleep(1.0)
    s.once()
    res["idle"] = {"derived": s.derived()}
    print("idle derived:", json.dumps(s.derived()), flush=True)
    print(s.text(), flush=True)
    out = os.path.join("gpurun_out", "pmc_probe.json")
    os.makedirs("gpurun_out", exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1, default=str)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
