"""Decode-shape small-kernel microbenchmark (run under rocprofv3 --kernel-trace --stats)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import reference as ref  # noqa: E402

ops.load_native(required=True)
T = int(sys.argv[1]) if len(sys.argv) > 1 else 256
dev = "cuda"
d, hq, hkv, D, BS, NB = 1024, 16, 8, 128, 32, 8192
x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
r = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
w = torch.ones(d, device=dev, dtype=torch.bfloat16)
qkv = torch.randn(T, (hq + 2 * hkv) * D, device=dev, dtype=torch.bfloat16)
q = torch.empty(T, hq, D, device=dev, dtype=torch.bfloat16)
kc = torch.zeros(NB, hkv, BS, D, device=dev, dtype=torch.bfloat16)
vc = torch.zeros(NB, hkv, BS // 8, D, 8, device=dev, dtype=torch.bfloat16)
pos = torch.randint(0, 4000, (T,), device=dev)
slots = torch.randperm(NB * BS, device=dev)[:T]
cs = ref.rope_cos_sin(4096, D, 1e6, device=dev)
qw = torch.ones(D, device=dev, dtype=torch.bfloat16)
gu = torch.randn(T, 6144, device=dev, dtype=torch.bfloat16)
noslots = torch.full_like(slots, -1)
# engine-like prefill slots: 512-token sequences, each in its own randomly placed blocks
_blocks = torch.randperm(NB, device=dev)
_tok = torch.arange(T, device=dev)
pslots = _blocks[_tok // BS] * BS + _tok % BS
# engine-like: 28 layers' caches, each written once per "step" (cold in L2)
L = 28
caches = [(torch.zeros(NB, hkv, BS, D, device=dev, dtype=torch.bfloat16),
           torch.zeros(NB, hkv, BS // 8, D, 8, device=dev, dtype=torch.bfloat16))
          for _ in range(L)]
qkvs = [torch.randn(T, (hq + 2 * hkv) * D, device=dev, dtype=torch.bfloat16) for _ in range(L)]
_layer = [0]


def layered():
    i = _layer[0] = (_layer[0] + 1) % L
    ops.qk_norm_rope_cache(qkvs[i], q, caches[i][0], caches[i][1], pos, pslots, cs, qw, qw, hq,
                           hkv, 1e-6)


fns = {
    "qk_rope_no_cache_write": lambda: ops.qk_norm_rope_cache(qkv, q, kc, vc, pos, noslots, cs,
                                                             qw, qw, hq, hkv, 1e-6),
    "qk_rope_28_layer_caches": layered,
    "qk_norm_rope_cache_prefill_slots": lambda: ops.qk_norm_rope_cache(
        qkv, q, kc, vc, pos, pslots, cs, qw, qw, hq, hkv, 1e-6),
    "rmsnorm": lambda: ops.rms_norm(x, w, 1e-6),
    "fused_add_rmsnorm": lambda: ops.fused_add_rms_norm(x, r, w, 1e-6),
    "qk_norm_rope_cache": lambda: ops.qk_norm_rope_cache(qkv, q, kc, vc, pos, slots, cs, qw, qw,
                                                         hq, hkv, 1e-6),
    "rope_cache_nonorm": lambda: ops.qk_norm_rope_cache(qkv, q, kc, vc, pos, slots, cs, None,
                                                        None, hq, hkv, 1e-6),
    "silu_and_mul": lambda: ops.silu_and_mul(gu),
}
for name, f in fns.items():
    f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(50):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(4):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:22s} T={T}: {e0.elapsed_time(e1) * 1000 / 200:7.2f} us/launch (graph, incl. boundary)")
