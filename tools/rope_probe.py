"""qk_norm_rope_cache (csrc/kernels/rope_cache.hip) on the headline prefill chunk: Qwen3-0.6B
heads (16 q / 8 kv, D = 128, q/k norm), 32 sequences x 512 tokens = 16,384 tokens into a
32-token-block paged cache; us per call (captured graph).

    python tools/rope_probe.py

Each shape is also timed in its serving form ("kv"): q rows left to the prefill attention
(q_rows = 0), the V tail on (one tail slot per sequence), 513-token prompts in the 32-sequence
case so every sequence ends in a partial V group.
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner as gt  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import reference as ref  # noqa: E402


def main():
    ops.load_native(required=True)
    dev = "cuda"
    hq, hkv, D, BS = 16, 8, 128, 32
    for nseq, L in ((32, 512), (32, 513), (4, 4096), (256, 1)):
        T = nseq * L
        nb = nseq * ((L + BS - 1) // BS) + 8
        qkv = torch.randn(T, (hq + 2 * hkv) * D, device=dev).to(torch.bfloat16)
        pos = torch.arange(L, device=dev).repeat(nseq).to(torch.int64)
        blocks = torch.randperm(nb, device=dev)
        per = (L + BS - 1) // BS
        slots = torch.cat([blocks[s * per + torch.arange(L, device=dev) // BS] * BS
                           + torch.arange(L, device=dev) % BS for s in range(nseq)]).to(torch.int64)
        cs = ref.rope_cos_sin(8192, D, 1e6, device=dev)
        qw = torch.randn(D, device=dev).to(torch.bfloat16)
        kw = torch.randn(D, device=dev).to(torch.bfloat16)
        kc = torch.zeros(nb, hkv, BS, D, device=dev, dtype=torch.bfloat16)
        vc = torch.zeros(nb, hkv, BS // 8, D, 8, device=dev, dtype=torch.bfloat16)
        q_out = torch.empty(T, hq, D, device=dev, dtype=torch.bfloat16)
        us = gt._timed(lambda i: ops.qk_norm_rope_cache(qkv, q_out, kc, vc, pos, slots, cs, qw, kw,
                                                        hq, hkv, 1e-6), 8)
        moved = T * (hq + 2 * hkv) * D * 2 + T * (hq + 2 * hkv) * D * 2
        vt = torch.zeros(nseq, hkv, 8, D, device=dev, dtype=torch.bfloat16)
        tsl = torch.arange(nseq, device=dev, dtype=torch.int32).repeat_interleave(L)
        us_kv = gt._timed(lambda i: ops.qk_norm_rope_cache(
            qkv, q_out, kc, vc, pos, slots, cs, qw, kw, hq, hkv, 1e-6, v_tail=vt, tail_slot=tsl,
            q_rows=0), 8)
        moved_kv = T * 2 * hkv * D * 2 * 2
        print(f"{nseq} x {L} ({T} tokens): {us:7.1f} us  ({moved / us / 1e6:5.2f} TB/s of qkv in + q/k/v out)"
              f" | kv {us_kv:7.1f} us ({moved_kv / us_kv / 1e6:5.2f} TB/s of k/v in + out)",
              flush=True)


if __name__ == "__main__":
    main()
