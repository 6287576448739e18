"""Workload for an HONEST FETCH_SIZE calibration: the counter is first read
on an INDEPENDENT streaming kernel whose HBM read bytes are known exactly, then the same
factor converts the production kernels' counts into bytes.

  calibration  akap::l2_prefetch_kernel streaming a 1 GiB bf16 buffer (4x the 256 MiB
               Infinity Cache: every byte comes from HBM) with 16-B-per-lane loads, 4 calls:
               known read = 1,073,741,824 B per call, nothing written
  production   the Qwen3-0.6B headline decode step at B=256 (all prompts 512 tokens, greedy,
               16 output tokens): paged_attn_decode_kernel, the fused GEMM chain, LM head --
               with their expected bytes per call printed for comparison (KV bytes streamed by
               one attention call; weight bytes of each projection)

Run under a counter pass, e.g.
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_cal -o run -- \
      python3 tools/pmc_calibrate.py
and reduce with tools/pmc_summary.py ... --calib 'l2_prefetch_kernel=1073741824'.
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams  # noqa: E402
from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine  # noqa: E402

CAL_BYTES = 1 << 30


def main():
    ops.load_native(required=True)
    buf = torch.empty(CAL_BYTES // 2, dtype=torch.bfloat16, device="cuda").normal_()
    torch.cuda.synchronize()
    for _ in range(4):
        ops.l2_prefetch([buf])
    torch.cuda.synchronize()
    del buf
    torch.cuda.empty_cache()

    eng = LLMEngine(EngineConfig(model="qwen3-0.6b", max_model_len=2048, max_num_seqs=256,
                                 max_num_batched_tokens=16384, block_size=32, device="cuda"))
    prompts = [[10 + (7 * i + j) % 150000 for j in range(512)] for i in range(256)]
    out_len = 16
    eng.generate(None, SamplingParams(max_tokens=out_len, temperature=0, ignore_eos=True),
                 prompt_ids=prompts)
    torch.cuda.synchronize()
    m = eng.runner.model
    hkv, D = m.hkv, m.D
    # decode step j (1..out_len-1) attends over 512 + j tokens per sequence (its own KV
    # written by the fused prologue first); K and V, bf16
    ctx = [512 + j for j in range(1, out_len)]
    kv_per_call = [256 * c * hkv * D * 2 * 2 for c in ctx]
    lw = m.layers[0]
    exp = {"calibration_kernel": "l2_prefetch_kernel", "calibration_bytes_per_call": CAL_BYTES,
           "attention_kv_bytes_per_call_mean": sum(kv_per_call) / len(kv_per_call),
           "attention_calls": len(kv_per_call) * len(m.layers),
           "weight_bytes": {n: getattr(lw, n).numel() * 2
                            for n in ("w_qkv", "w_o", "w_gate_up", "w_down")},
           "lm_head_bytes": m.lm_head.numel() * 2,
           "activation_bytes_M256": {n: 256 * getattr(lw, n).shape[1] * 2
                                     for n in ("w_qkv", "w_o", "w_gate_up", "w_down")}}
    print("EXPECTED " + json.dumps(exp), flush=True)


if __name__ == "__main__":
    main()
