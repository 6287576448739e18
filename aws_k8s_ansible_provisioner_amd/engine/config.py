"""Engine / sampling configuration (argument names mirror the vLLM OpenAI server so the
llm-d style manifests and the reference's smoke test keep working)."""
from __future__ import annotations

import dataclasses
from typing import Optional


@dataclasses.dataclass
class EngineConfig:
    model: str = "qwen3-0.6b"
    served_model_name: Optional[str] = None
    max_model_len: int = 4096
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 16384
    block_size: int = 32
    gpu_memory_utilization: float = 0.90
    num_gpu_blocks: Optional[int] = None      # override the memory-derived block count
    kv_cache_max_gib: Optional[float] = None  # cap on the memory-derived KV cache size
    enable_prefix_caching: bool = True
    enforce_eager: bool = False               # disable hipGraph decode
    cuda_graph_max_bs: Optional[int] = None   # largest captured decode batch
    tensor_parallel_size: int = 1
    seed: int = 0
    device: str = "auto"                      # "auto" | "cuda" | "cpu"
    load_format: str = "random"               # "random" | "safetensors"
    weights_path: Optional[str] = None
    chat_template: Optional[str] = None
    kv_role: str = "both"                     # "both" | "prefill" | "decode" (P/D)
    kv_cache_dtype: str = "auto"              # "auto" (model dtype, bf16) | "fp8" (e4m3fn)
    init_std: float = 0.02                    # random-init weight scale
    shard_init: str = "per_rank"              # "per_rank" | "full" (identical logical weights for any TP)
    mixed_batching: bool = True               # decodes + prefill chunks in one step
    mix_backlog_steps: int = 1                # ... unless more prefill is queued than this
    max_decode_stall_steps: int = 8           #     many steps' budget (burst: TTFT first),
    #                                           for at most this many steps in a row
    held_kv_ttl_s: float = 120.0              # P/D prefill: free un-pulled held KV after this
    gc_freeze: bool = True                    # gc.freeze() the start-up heap (no full-GC stalls)
    # decode lookahead: queue decode step N+1 (inputs gathered on the GPU from step N's
    # samples) before waiting for step N, so host bookkeeping and the graph launch overlap
    # the GPU (single-rank engines with hipGraphs; AKAP_ASYNC_DECODE=0 disables)
    async_decode: bool = True

    def __post_init__(self) -> None:
        # the K cache stores each 32-token chunk in MFMA-fragment order (ops/reference.py)
        if self.block_size <= 0 or self.block_size % 32:
            raise ValueError(f"block_size must be a multiple of 32, got {self.block_size}")
        if self.kv_cache_dtype not in ("auto", "bf16", "bfloat16", "fp8", "fp8_e4m3"):
            raise ValueError(f"kv_cache_dtype must be auto or fp8, got {self.kv_cache_dtype}")

    def resolved_device(self) -> str:
        if self.device != "auto":
            return self.device
        import torch

        return "cuda" if torch.cuda.is_available() else "cpu"


@dataclasses.dataclass
class SamplingParams:
    max_tokens: int = 16
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    min_tokens: int = 0
    seed: Optional[int] = None
    stop_token_ids: list = dataclasses.field(default_factory=list)
    stop: list = dataclasses.field(default_factory=list)  # stop strings (post-detokenize)
    ignore_eos: bool = False
    logprobs: Optional[int] = None           # return the sampled token's log-prob
    n: int = 1
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    repetition_penalty: float = 1.0

    @property
    def has_penalties(self) -> bool:
        return (self.presence_penalty != 0.0 or self.frequency_penalty != 0.0
                or self.repetition_penalty != 1.0)

    def normalized(self) -> "SamplingParams":
        p = dataclasses.replace(self)
        if p.top_k is None or p.top_k < 0:
            p.top_k = 0
        if p.top_p is None or p.top_p <= 0:
            p.top_p = 1.0
        if p.temperature is None:
            p.temperature = 1.0
        if p.temperature < 1e-5:
            p.temperature = 0.0
        if p.repetition_penalty is None or p.repetition_penalty <= 0:
            p.repetition_penalty = 1.0
        p.presence_penalty = float(p.presence_penalty or 0.0)
        p.frequency_penalty = float(p.frequency_penalty or 0.0)
        return p
