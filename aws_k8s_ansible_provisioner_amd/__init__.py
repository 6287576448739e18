"""MI355X-native one-command K8s provisioner + llm-d-compatible serving stack.

Subpackages:
  ops/       gfx950 HIP kernels (torch.ops.akap) + PyTorch references
  models/    Qwen3 / Llama-3 / Mixtral decoder on those kernels
  engine/    C++ scheduler + paged KV block manager, model runner, hipGraph decode
  parallel/  torch.distributed over RCCL/xGMI: TP, EP all-to-all, P/D KV transfer
  server/    OpenAI-compatible HTTP server (vLLM-compatible args / metrics)
  gateway/   inference gateway + endpoint picker (least-loaded / prefix / P-D)
  exporter/  amd-smi GPU metrics exporter (DCGM-compatible aliases)
  utils/     tokenizer, chat templates, metrics, tracing
"""
__version__ = "0.1.0"
