"""Prefill GEMMs (hipBLASLt through F.linear) with and without PyTorch-ROCm TunableOp: how much
does tuning the library's solution per shape buy at prefill sizes?

    python tools/prefill_gemm_tunableop.py [--M 16384]
"""
import argparse
import os

import torch
import torch.nn.functional as F

SHAPES = {
    "qwen3": [("qkv", 4096, 1024), ("o", 1024, 2048), ("gate_up", 6144, 1024), ("down", 1024, 3072)],
    "llama8b": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096),
                ("down", 4096, 14336)],
}


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[16384, 9000])
    a = ap.parse_args()
    tun = torch.cuda.tunable
    tun.set_filename(os.path.join("/tmp", "tunableop_probe.csv"))
    for model, shapes in SHAPES.items():
        for M in a.M:
            tot0 = tot1 = 0.0
            for name, N, K in shapes:
                x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
                tun.enable(False)
                t0 = timed(lambda: F.linear(x, w))
                tun.enable(True)
                tun.tuning_enable(True)
                tun.set_max_tuning_iterations(20)
                F.linear(x, w)  # tunes this shape
                tun.tuning_enable(False)
                t1 = timed(lambda: F.linear(x, w))
                tun.enable(False)
                fl = 2.0 * M * N * K
                tot0 += t0
                tot1 += t1
                print(f"{model:8s} M={M:6d} {name:8s} N={N:6d} K={K:6d}: default {t0:8.1f} us "
                      f"({fl / t0 / 1e6:6.0f} TF)  tuned {t1:8.1f} us ({fl / t1 / 1e6:6.0f} TF)",
                      flush=True)
            print(f"{model} M={M}: per layer default {tot0:.0f} us, tuned {tot1:.0f} us", flush=True)


if __name__ == "__main__":
    main()
