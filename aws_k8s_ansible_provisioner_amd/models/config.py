"""Model architecture configs (random-init friendly: no checkpoint download needed).

The registry holds the exact shapes of the model families the reference stack
serves or the north star names (Qwen3-0.6B is what ``llm-d-deploy.yaml:118`` deploys;
Llama-3-8B / 70B and Mixtral-8x7B are the disaggregated, TP=8 and EP configs of
BASELINE.json), plus tiny variants for CPU tests.  A HF ``config.json`` can also be
loaded (``from_hf_dict``) when real weights are mounted from the model PVC.
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Optional


@dataclasses.dataclass
class ModelConfig:
    name: str
    hf_id: str
    arch: str  # "qwen3" | "llama" | "mixtral" | "qwen3_moe"
    vocab_size: int
    hidden_size: int
    intermediate_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int = 128
    rms_eps: float = 1e-6
    rope_theta: float = 10000.0
    rope_scaling: Optional[dict] = None
    max_position: int = 32768
    tie_embeddings: bool = False
    qk_norm: bool = False
    num_experts: int = 0
    experts_per_token: int = 0
    moe_renormalize: bool = True  # top-k router weights renormalised to sum 1 (norm_topk_prob)
    bos_id: int = 1
    eos_id: int = 2
    dtype: str = "bfloat16"

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    @property
    def gqa_group(self) -> int:
        return self.num_heads // self.num_kv_heads

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    def kv_bytes_per_token(self, tp: int = 1) -> int:
        return self.num_layers * 2 * max(1, self.num_kv_heads // tp) * self.head_dim * 2

    def num_params(self) -> int:
        d, f, L = self.hidden_size, self.intermediate_size, self.num_layers
        attn = d * (self.q_size + 2 * self.kv_size) + self.q_size * d
        mlp = 3 * d * f * (self.num_experts if self.is_moe else 1)
        router = d * self.num_experts if self.is_moe else 0
        emb = self.vocab_size * d * (1 if self.tie_embeddings else 2)
        return L * (attn + mlp + router + 2 * d) + emb + d

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    @staticmethod
    def from_hf_dict(name: str, d: dict) -> "ModelConfig":
        mt = d.get("model_type", "llama")
        arch = {"qwen3": "qwen3", "mixtral": "mixtral", "qwen3_moe": "qwen3_moe"}.get(mt, "llama")
        heads = d["num_attention_heads"]
        moe_ffn = d.get("moe_intermediate_size") if arch == "qwen3_moe" else None
        return ModelConfig(
            name=name, hf_id=name, arch=arch, vocab_size=d["vocab_size"],
            hidden_size=d["hidden_size"], intermediate_size=moe_ffn or d["intermediate_size"],
            num_layers=d["num_hidden_layers"], num_heads=heads,
            num_kv_heads=d.get("num_key_value_heads", heads),
            head_dim=d.get("head_dim") or d["hidden_size"] // heads,
            rms_eps=d.get("rms_norm_eps", 1e-6), rope_theta=d.get("rope_theta", 10000.0),
            rope_scaling=d.get("rope_scaling"),
            max_position=d.get("max_position_embeddings", 32768),
            tie_embeddings=d.get("tie_word_embeddings", False),
            qk_norm=arch in ("qwen3", "qwen3_moe"),
            num_experts=d.get("num_local_experts", d.get("num_experts", 0)),
            experts_per_token=d.get("num_experts_per_tok", 0),
            moe_renormalize=bool(d.get("norm_topk_prob", True)),
            bos_id=d.get("bos_token_id", 1) or 1,
            eos_id=(d.get("eos_token_id", 2) if not isinstance(d.get("eos_token_id"), list)
                    else d["eos_token_id"][0]),
        )


_REGISTRY: dict[str, ModelConfig] = {}


def register(cfg: ModelConfig) -> ModelConfig:
    _REGISTRY[cfg.name] = cfg
    _REGISTRY[cfg.hf_id.lower()] = cfg
    return cfg


# Qwen3-0.6B -- the model the reference deploys (llm-d-deploy.yaml:118, llm-d-test.yaml:7)
QWEN3_0_6B = register(ModelConfig(
    name="qwen3-0.6b", hf_id="Qwen/Qwen3-0.6B", arch="qwen3", vocab_size=151936,
    hidden_size=1024, intermediate_size=3072, num_layers=28, num_heads=16, num_kv_heads=8,
    head_dim=128, rms_eps=1e-6, rope_theta=1_000_000.0, max_position=40960,
    tie_embeddings=True, qk_norm=True, bos_id=151643, eos_id=151645))

LLAMA3_8B = register(ModelConfig(
    name="llama-3-8b", hf_id="meta-llama/Meta-Llama-3-8B-Instruct", arch="llama",
    vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_layers=32,
    num_heads=32, num_kv_heads=8, head_dim=128, rms_eps=1e-5, rope_theta=500000.0,
    max_position=8192, bos_id=128000, eos_id=128009))

LLAMA3_70B = register(ModelConfig(
    name="llama-3-70b", hf_id="meta-llama/Meta-Llama-3-70B-Instruct", arch="llama",
    vocab_size=128256, hidden_size=8192, intermediate_size=28672, num_layers=80,
    num_heads=64, num_kv_heads=8, head_dim=128, rms_eps=1e-5, rope_theta=500000.0,
    max_position=8192, bos_id=128000, eos_id=128009))

# Llama-3-70B's real layer widths (d 8192, 64/8 heads, ffn 28672, vocab 128256) at 4 layers:
# the TP=4 / TP=8 decode collectives at their production message sizes (B=256 x 8192 bf16 =
# 4 MiB per all-reduce) on one GPU, multi-process
LLAMA3_70B_L4 = register(ModelConfig(
    name="llama-3-70b-l4", hf_id="test/llama-3-70b-l4", arch="llama",
    vocab_size=128256, hidden_size=8192, intermediate_size=28672, num_layers=4,
    num_heads=64, num_kv_heads=8, head_dim=128, rms_eps=1e-5, rope_theta=500000.0,
    max_position=8192, bos_id=128000, eos_id=128009))

MIXTRAL_8X7B = register(ModelConfig(
    name="mixtral-8x7b", hf_id="mistralai/Mixtral-8x7B-Instruct-v0.1", arch="mixtral",
    vocab_size=32000, hidden_size=4096, intermediate_size=14336, num_layers=32,
    num_heads=32, num_kv_heads=8, head_dim=128, rms_eps=1e-5, rope_theta=1_000_000.0,
    max_position=32768, num_experts=8, experts_per_token=2, bos_id=1, eos_id=2))

# Qwen3 mixture-of-experts: 128 fine-grained experts, 8 per token (3.3B of 30.5B parameters
# active); every layer MoE, q/k RMSNorm like the dense Qwen3
QWEN3_30B_A3B = register(ModelConfig(
    name="qwen3-30b-a3b", hf_id="Qwen/Qwen3-30B-A3B", arch="qwen3_moe", vocab_size=151936,
    hidden_size=2048, intermediate_size=768, num_layers=48, num_heads=32, num_kv_heads=4,
    head_dim=128, rms_eps=1e-6, rope_theta=1_000_000.0, max_position=40960, qk_norm=True,
    num_experts=128, experts_per_token=8, bos_id=151643, eos_id=151645))

# tiny shapes for CPU tests / smoke (same code paths, seconds to run)
TINY_QWEN3 = register(ModelConfig(
    name="tiny-qwen3", hf_id="test/tiny-qwen3", arch="qwen3", vocab_size=512,
    hidden_size=256, intermediate_size=512, num_layers=2, num_heads=4, num_kv_heads=2,
    head_dim=128, rope_theta=1_000_000.0, max_position=4096, tie_embeddings=True,
    qk_norm=True, bos_id=1, eos_id=2))

TINY_LLAMA = register(ModelConfig(
    name="tiny-llama", hf_id="test/tiny-llama", arch="llama", vocab_size=512,
    hidden_size=256, intermediate_size=512, num_layers=2, num_heads=4, num_kv_heads=2,
    head_dim=128, rope_theta=500000.0, max_position=4096, bos_id=1, eos_id=2))

TINY_MIXTRAL = register(ModelConfig(
    name="tiny-mixtral", hf_id="test/tiny-mixtral", arch="mixtral", vocab_size=512,
    hidden_size=256, intermediate_size=256, num_layers=2, num_heads=4, num_kv_heads=2,
    head_dim=128, rope_theta=1_000_000.0, max_position=4096, num_experts=4,
    experts_per_token=2, bos_id=1, eos_id=2))


TINY_QWEN3_MOE = register(ModelConfig(
    name="tiny-qwen3-moe", hf_id="test/tiny-qwen3-moe", arch="qwen3_moe", vocab_size=512,
    hidden_size=256, intermediate_size=256, num_layers=2, num_heads=4, num_kv_heads=2,
    head_dim=128, rope_theta=1_000_000.0, max_position=4096, qk_norm=True, num_experts=16,
    experts_per_token=4, bos_id=1, eos_id=2))


# the real multi-GPU layouts at world size 8: Llama-3-70B's 8 KV heads (one per TP rank, GQA
# 8) and Mixtral's 8 experts (one per EP rank)
TINY_LLAMA_KV8 = register(ModelConfig(
    name="tiny-llama-kv8", hf_id="test/tiny-llama-kv8", arch="llama", vocab_size=512,
    hidden_size=256, intermediate_size=512, num_layers=2, num_heads=16, num_kv_heads=8,
    head_dim=128, rope_theta=500000.0, max_position=4096, bos_id=1, eos_id=2))

TINY_MIXTRAL8 = register(ModelConfig(
    name="tiny-mixtral8", hf_id="test/tiny-mixtral8", arch="mixtral", vocab_size=512,
    hidden_size=256, intermediate_size=256, num_layers=2, num_heads=16, num_kv_heads=8,
    head_dim=128, rope_theta=1_000_000.0, max_position=4096, num_experts=8,
    experts_per_token=2, bos_id=1, eos_id=2))


def get_config(name: str) -> ModelConfig:
    """Resolve a registry name, HF id, or a directory holding a HF config.json."""
    if os.path.isdir(name) and os.path.exists(os.path.join(name, "config.json")):
        with open(os.path.join(name, "config.json")) as f:
            return ModelConfig.from_hf_dict(name, json.load(f))
    key = name.lower()
    if key in _REGISTRY:
        return _REGISTRY[key]
    raise KeyError(f"unknown model {name!r}; known: {sorted(set(c.name for c in _REGISTRY.values()))}")


def list_models() -> list[str]:
    return sorted(set(c.name for c in _REGISTRY.values()))
