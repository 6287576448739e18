"""How much of each served decode GEMM is the cold weight fetch?  (round 6)

The Qwen3-0.6B decode layer chain at M = 256 runs four fused GEMM launches (the variants the
tuner picks: qkv register ring s1p4 + ss_in scale, o kgemm k32 + residual/norm epilogue,
gate_up LDS-DMA 64x128 deep ring + SwiGLU, down kgemm k32 + residual/norm).  In serving their
weights are cold: the 28 layers' weights (868 MB) and each layer's KV stream (~335 MB at
B = 256, ctx ~640) overflow the 256 MB MALL between two uses.  This probe times each launch
with its weights
  cold : rotating over 28 distinct layer copies (the tuner's measurement, = serving)
  mall : rotating over 4 copies with a 96 MB read between launches (weights in MALL, not L2;
         reported as t(flush + gemm) - t(flush))
  warm : the same copy every launch (L2 + MALL resident)
If mall << cold, moving each layer's weights into the MALL ahead of its GEMM (a prefetch
overlapped with the HBM-bound attention) is the lever; if not, the chain is bound by its
own L2 -> CU ingress.
python tools/weight_warmth_probe.py [--M 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops.gemm_tuner import _timed  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=256)
    ap.add_argument("--layers", type=int, default=28)
    a = ap.parse_args()
    ops.load_native(required=True)
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    M, L = a.M, a.layers
    d, F = 1024, 3072
    shapes = {"qkv": (4096, d), "o": (d, 2048), "gate_up": (2 * F, d), "down": (d, F)}
    g = torch.Generator(device=dev).manual_seed(0)
    W = {k: [torch.randn(n, kk, device=dev, dtype=bf, generator=g) * 0.02 for _ in range(L)]
         for k, (n, kk) in shapes.items()}
    ln = torch.rand(d, device=dev, dtype=bf) + 0.5
    ss = torch.full((M,), float(d), device=dev)
    ss_o = torch.zeros(M, device=dev)
    a_o = torch.empty(M, d, device=dev, dtype=bf)
    res = torch.randn(M, d, device=dev, dtype=bf)
    xs = {k: torch.randn(M, kk, device=dev, dtype=bf) * 0.1 for k, (n, kk) in shapes.items()}
    out = {"qkv": torch.empty(M, 4096, device=dev, dtype=bf),
           "gate_up": torch.empty(M, F, device=dev, dtype=bf)}
    flush = torch.empty(48 << 20, device=dev, dtype=bf)  # 96 MB > the 8 x 4 MB of L2
    flush.normal_()
    fl_out = torch.empty((), device=dev, dtype=torch.float32)

    def call(k, w):
        if k == "qkv":
            ops.dgemm(xs[k], w, splitk=1, pf=4, out=out[k], ss_in=ss)
        elif k == "gate_up":
            ops.dgemm(xs[k], w, splitk=1, bn=128, ns=8, out=out[k], epi=ops.EPI_SILU, ss_in=ss)
        else:  # o / down: kgemm 32-row tiles, residual + next-norm epilogue
            torch.ops.akap.kgemm(res, xs[k], w, 32, ops.EPI_RESNORM, 1e-6, None, ss_o, a_o, ln)

    def fl():
        torch.sum(flush, dim=(0,), dtype=torch.float32, out=fl_out)

    print(f"M={M}, {L} layer copies; us per launch (best of 3 graph-replay windows)")
    print(f"{'gemm':8s} {'MB':>6s} {'cold':>7s} {'mall':>7s} {'warm':>7s}  flush")
    for k, ws in W.items():
        mb = ws[0].numel() * 2 / 1e6
        t_cold = _timed(lambda i: call(k, ws[i % L]), L)
        t_warm = _timed(lambda i: call(k, ws[0]), L)
        t_fl = _timed(lambda i: fl(), L)
        t_flg = _timed(lambda i: (fl(), call(k, ws[i % 4])), L)
        print(f"{k:8s} {mb:6.1f} {t_cold:7.2f} {t_flg - t_fl:7.2f} {t_warm:7.2f}  {t_fl:.2f}",
              flush=True)
    # the down projection's split-K forms (VERDICT r5 "Step A"): slabs + the row reduce launch,
    # the same slices combined inside the launch (dgemm SPL 2), and kgemm (K split inside the
    # workgroup); cold weights, residual + next-norm epilogue
    wd = W["down"]
    ws4 = torch.empty(4 * M * d, device=dev, dtype=torch.float32)
    ws4i = torch.empty(ops.gdgemm_ws_floats(M, d, 4, 64, 64), device=dev, dtype=torch.float32)
    cnt = ops.gemm_counters(dev)
    forms = {
        "s4p4 slabs + reduce": lambda i: torch.ops.akap.dgemm(
            res, xs["down"], wd[i % L], ws4, 0, 4, 4, None, None, None, 1e-6, ops.EPI_RESNORM,
            None, ss_o, a_o, ln, 0),
        "s4p4 in-launch": lambda i: torch.ops.akap.dgemm(
            res, xs["down"], wd[i % L], ws4i, 0, 4, 4, None, None, None, 1e-6, ops.EPI_RESNORM,
            None, ss_o, a_o, ln, 0, 0, cnt, 64),
        "k32": lambda i: torch.ops.akap.kgemm(res, xs["down"], wd[i % L], 32, ops.EPI_RESNORM,
                                              1e-6, None, ss_o, a_o, ln),
    }
    for name, fn in forms.items():
        print(f"down {name:22s} {_timed(fn, L):7.2f} us", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
