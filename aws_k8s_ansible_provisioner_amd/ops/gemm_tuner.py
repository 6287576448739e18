"""Per-shape decode-GEMM dispatch: hipBLASLt vs the hand-written MFMA GEMM (csrc/kernels/
gemm.hip) at its best split-K, chosen by measurement at engine start.

Decode GEMMs read every layer's weights once per step, cold (the KV stream has evicted
them), and at M = batch they are latency/issue bound rather than bandwidth bound, so the
winner depends on (M, N, K): measured on MI355X, Llama-3-8B's down projection at M=128 is
49 us with the MFMA kernel at split-K 8 vs 75 us in hipBLASLt, while hipBLASLt wins the
wide gate|up projection (`profiles/r1_gemm_splitk_sweep.log`).  PyTorch TunableOp cannot
make this choice: it only ranks hipBLASLt/rocBLAS solutions, and it times them on warm
weights.

The tuner times each candidate on the model's REAL per-layer weights, rotating through
all layers inside one captured hipGraph (so every call sees cold weights, as in a decode
step), and records the winner in the plan `ops.linear` consults.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

Choice = tuple  # ("torch",) | ("hip", splitk)
_PLAN: dict = {}


def plan() -> dict:
    return _PLAN


def lookup(M: int, N: int, K: int) -> Optional[Choice]:
    return _PLAN.get((M, N, K))


def _timed(fn, n: int) -> float:
    """us per call of fn(i), i < n, measured on a captured graph replay."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(min(n, 2)):
            fn(i)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    g.replay()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / (2 * n)


def tune(M: int, weights: Sequence[torch.Tensor], splits=(1, 2, 4, 8, 16),
         margin: float = 0.03) -> Choice:
    """Pick the fastest way to compute x[M, K] @ w.T for these same-shape weights.
    hipBLASLt is kept unless the MFMA kernel is more than `margin` faster."""
    from . import gemm_counters  # noqa: F401  (ensures the native library is loaded)

    w0 = weights[0]
    N, K = w0.shape
    dev = w0.device
    x = torch.randn(M, K, device=dev, dtype=w0.dtype) * 0.1
    y = torch.empty(M, N, device=dev, dtype=w0.dtype)
    n = len(weights)
    best: Choice = ("torch",)
    t_best = _timed(lambda i: torch.nn.functional.linear(x, weights[i % n]), n)
    t_torch = t_best
    for s in splits:
        if K // s < 256 or K % (64 * s):
            continue
        ws = torch.empty(max(1, s * M * N), device=dev, dtype=torch.float32)
        t = _timed(lambda i: torch.ops.akap.gemm(y, x, weights[i % n], ws, s), n)
        if t < t_best:
            best, t_best = ("hip", s), t
    if best[0] == "hip" and t_best > t_torch * (1.0 - margin):
        best = ("torch",)
    _PLAN[(M, N, K)] = best
    return best


def tune_model(model, Ms: Sequence[int], log=print) -> dict:
    """Tune every dense projection shape of `model` (per layer type) for each M."""
    groups = {}
    for lw in model.layers:
        for name in ("w_qkv", "w_o", "w_gate_up", "w_down"):
            w = getattr(lw, name, None)
            if w is not None:
                groups.setdefault((name, tuple(w.shape)), []).append(w)
    summary = {}
    for M in Ms:
        for (name, shape), ws in groups.items():
            summary[(M, name)] = tune(M, ws)
    wins = {k: v for k, v in summary.items() if v[0] == "hip"}
    log(f"[gemm-tuner] {len(summary)} decode GEMM shapes, MFMA kernel chosen for "
        f"{len(wins)}: " + ", ".join(f"M={m} {n} s{c[1]}" for (m, n), c in sorted(wins.items())))
    return summary
