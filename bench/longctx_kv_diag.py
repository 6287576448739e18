"""Long-prompt KV-cache check: after the chunked prefill of a T-token prompt, compare layer 0's
paged K/V cache (written by the GPU prefill kernels) with K/V recomputed densely from the same
weights; print the worst error per 512-position bucket."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams  # noqa: E402
from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import reference as ref  # noqa: E402

T = int(os.environ.get("DIAG_T", "7000"))
eng = LLMEngine(EngineConfig(model="qwen3-0.6b", device="cuda", max_model_len=16384,
                             max_num_seqs=4, cuda_graph_max_bs=4,
                             max_num_batched_tokens=int(os.environ.get("DIAG_CHUNK", "1024")),
                             block_size=32, num_gpu_blocks=600, init_std=0.05),
                log=lambda *a: None)
prompt = [int(x) for x in torch.randint(5, 1000, (T,), generator=torch.Generator().manual_seed(0))]
name = eng.add_request(None, None, SamplingParams(max_tokens=4, temperature=0, ignore_eos=True),
                       prompt_ids=prompt, stream=True)
iid = eng.by_name[name]
while True:
    outs = eng.step()
    if any(o.req_id == name for o in outs):
        break
torch.cuda.synchronize()
bt = torch.tensor(eng.sched.block_table(iid), dtype=torch.int32)
m = eng.runner.model
lw = m.layers[0]
D, hq, hkv = m.D, m.hq, m.hkv
t = torch.tensor(prompt, device="cuda")
x = m.embed[t].float()
h = ref.rms_norm(x.bfloat16(), lw.ln1, m.cfg.rms_eps).float()
qkv = (h @ lw.w_qkv.float().t())
k = qkv[:, hq * D:(hq + hkv) * D].view(T, hkv, D)
v = qkv[:, (hq + hkv) * D:].view(T, hkv, D)
if lw.k_norm is not None:
    k = ref.rms_norm(k.bfloat16(), lw.k_norm, m.cfg.rms_eps).float()
k = ref.apply_rope(k, torch.arange(T, device="cuda"), m.cos_sin)
K, V = ref.gather_kv(eng.runner.k_caches[0].cpu(), eng.runner.v_caches[0].cpu(), bt, T)
ek = (K.float() - k.cpu()).abs().amax(dim=(1, 2))
ev = (V.float() - v.cpu()).abs().amax(dim=(1, 2))
print(f"T={T} blocks={bt.tolist()[:4]}..{bt.tolist()[-3:]}")
for b0 in range(0, T, 512):
    print(f"  pos {b0:5d}-{min(T, b0 + 512) - 1:5d}: max|dK| {ek[b0:b0 + 512].max():.4f}"
          f"  max|dV| {ev[b0:b0 + 512].max():.4f}", flush=True)
