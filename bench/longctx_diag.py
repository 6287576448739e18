"""Long-context decode diagnostic: Qwen3-0.6B shapes, an 8k-token prompt, greedy decode;
prints each generated token's gap to the dense fp32 reference's argmax (in logit std units)
and the decode split-KV plan.  Run under different AKAP_* switches to bisect a mismatch."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams  # noqa: E402
from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine  # noqa: E402
from aws_k8s_ansible_provisioner_amd.models.reference_forward import dense_logits  # noqa: E402

T = int(os.environ.get("DIAG_T", "8000"))
eager = os.environ.get("DIAG_EAGER", "0") == "1"
eng = LLMEngine(EngineConfig(model=os.environ.get("DIAG_MODEL", "qwen3-0.6b"),
                             device=os.environ.get("DIAG_DEVICE", "cuda"),
                             max_model_len=int(os.environ.get("DIAG_MAXLEN", "16384")),
                             max_num_seqs=4, cuda_graph_max_bs=4, max_num_batched_tokens=1024,
                             block_size=32, num_gpu_blocks=600, init_std=0.05,
                             enforce_eager=eager), log=lambda *a: None)
prompt = [int(x) for x in torch.randint(5, 1000, (T,), generator=torch.Generator().manual_seed(0))]
out = eng.generate(None, SamplingParams(max_tokens=6, temperature=0, ignore_eos=True),
                   prompt_ids=[prompt])[0]
logits = dense_logits(eng.runner.model, prompt + out.output_ids).float()
gaps = []
for i, tok in enumerate(out.output_ids):
    row = logits[T - 1 + i]
    gaps.append(round(((row.max() - row[tok]) / (row.std() + 1e-6)).item(), 3))
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith(("AKAP_", "DIAG_")))
print(f"[{tag}] T={T} parts={eng.runner.decode_partitions(1)} tokens={out.output_ids} "
      f"gaps={gaps}", flush=True)
