"""Narrow down a TP=1 GPU divergence from the dense reference (tiny-llama, prompt [100, 101])."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams  # noqa: E402
from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine  # noqa: E402
from aws_k8s_ansible_provisioner_amd.models.reference_forward import dense_logits  # noqa: E402


def run(tag, prompts, **kw):
    cfg = dict(model="tiny-llama", device="cuda", max_model_len=256, max_num_seqs=8,
               max_num_batched_tokens=64, block_size=32, num_gpu_blocks=96, init_std=0.15,
               enforce_eager=True, shard_init="full")
    cfg.update(kw)
    eng = LLMEngine(EngineConfig(**cfg), log=lambda *a: None)
    outs = eng.generate(None, SamplingParams(max_tokens=6, temperature=0, ignore_eos=True),
                        prompt_ids=prompts)
    for p, o in zip(prompts, outs):
        seq = list(p) + list(o.output_ids)
        lg = dense_logits(eng.runner.model, seq).float().cpu()
        tf = [int(lg[len(p) - 1 + i].argmax()) for i in range(len(o.output_ids))]
        ok = "OK " if tf == list(o.output_ids) else "BAD"
        gaps = []
        for i, t in enumerate(o.output_ids):
            row = lg[len(p) - 1 + i]
            gaps.append(round(float((row.max() - row[t]) / (row.std() + 1e-6)), 4))
        print(f"{ok} {tag:40s} len {len(p):3d} got {o.output_ids} dense {tf} gap/std {gaps}",
              flush=True)


if __name__ == "__main__":
    P = [[100, 101]]
    run("eager full 0.15", P)
    if os.environ.get("ONLY_FIRST"):
        sys.exit(0)
    run("eager default-init 0.15", P, shard_init="per_rank")
    run("eager full 0.10", P, init_std=0.1)
    run("graphs full 0.15", P, enforce_eager=False)
    run("eager full 0.15 bs16", P, block_size=16) if False else None
    run("eager full 0.15 prompt 100,101,102", [[100, 101, 102]])
    run("eager full 0.15 prompt 5,6", [[5, 6]])
    run("eager full 0.15 prompt 100", [[100]])
    run("eager full 0.15 qwen3", P, model="tiny-qwen3")
