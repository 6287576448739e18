"""HF-named checkpoint loading (B3: the model-PVC loader): q/k/v -> fused w_qkv, gate/up ->
fused w_gate_up, Mixtral experts -> w13/w2, and the TP / EP sharding of all of them.  No
download: the state dict is exported from a tiny model, written as safetensors, and loaded
into differently-seeded models at tp=1 and (2 gloo processes) tp=2; every path must
reproduce the source model's logits / greedy tokens."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine
from aws_k8s_ansible_provisioner_amd.models.config import get_config
from aws_k8s_ansible_provisioner_amd.models.reference_forward import dense_logits
from aws_k8s_ansible_provisioner_amd.models.transformer import DecoderLM

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROMPTS = [list(range(5, 40)), [100, 101], [9, 9, 9]]


def _export(model, tmp_path):
    from safetensors.torch import save_file

    src = DecoderLM(get_config(model), "cpu", seed=11, max_model_len=256, init_std=0.15)
    sd = src.hf_state_dict()
    d = tmp_path / model
    d.mkdir()
    save_file({k: v.contiguous() for k, v in sd.items()}, str(d / "model.safetensors"))
    return src, sd, str(d)


@pytest.mark.parametrize("model", ["tiny-qwen3", "tiny-llama", "tiny-mixtral", "tiny-qwen3-moe"])
def test_hf_names_round_trip_tp1(model, tmp_path):
    src, sd, _ = _export(model, tmp_path)
    names = set(sd)
    assert "model.layers.0.self_attn.q_proj.weight" in names
    if get_config(model).arch == "qwen3_moe":
        assert "model.layers.0.mlp.experts.1.up_proj.weight" in names
        assert "model.layers.0.mlp.gate.weight" in names
    elif get_config(model).is_moe:
        assert "model.layers.0.block_sparse_moe.experts.1.w3.weight" in names
    else:
        assert "model.layers.0.mlp.gate_proj.weight" in names
    dst = DecoderLM(get_config(model), "cpu", seed=99, max_model_len=256, init_std=0.15)
    assert not torch.equal(dst.layers[0].w_qkv, src.layers[0].w_qkv)
    dst.load_state_dict(sd)
    for a, b in zip(src.layers, dst.layers):
        assert torch.equal(a.w_qkv, b.w_qkv) and torch.equal(a.w_o, b.w_o)
    for p in PROMPTS:
        assert torch.equal(dense_logits(src, p), dense_logits(dst, p))


CHILD = r"""
import json, os, sys
sys.path.insert(0, os.environ["ROOT"])
from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
from aws_k8s_ansible_provisioner_amd.parallel.tp_worker import make_tp_engine
ecfg = EngineConfig(model=os.environ["MODEL"], device="cpu", max_model_len=256, max_num_seqs=8,
                    max_num_batched_tokens=32, block_size=32, num_gpu_blocks=96,
                    tensor_parallel_size=2, seed=77, load_format="safetensors",
                    weights_path=os.environ["WEIGHTS"])
eng, bc = make_tp_engine(ecfg, backend="gloo", log=lambda *a: None)
if eng is not None:
    outs = eng.generate(None, SamplingParams(max_tokens=6, temperature=0, ignore_eos=True),
                        prompt_ids=json.loads(os.environ["PROMPTS"]))
    bc.shutdown()
    print("RESULT " + json.dumps([o.output_ids for o in outs]), flush=True)
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("model,moe_mode", [("tiny-llama", "tp"), ("tiny-qwen3", "tp"),
                                            ("tiny-mixtral", "tp"), ("tiny-mixtral", "ep"),
                                            ("tiny-qwen3-moe", "tp"), ("tiny-qwen3-moe", "ep")])
def test_hf_checkpoint_sharded_load_tp2(model, moe_mode, tmp_path):
    """The same safetensors checkpoint loaded by a tp=2 engine (each rank takes its q/kv-head,
    ffn-row, vocab and expert shards) generates the tokens of the tp=1 engine that loaded it."""
    src, sd, wdir = _export(model, tmp_path)
    ref = LLMEngine(EngineConfig(model=model, device="cpu", max_model_len=256, max_num_seqs=8,
                                 max_num_batched_tokens=32, block_size=32, num_gpu_blocks=96,
                                 seed=5, load_format="safetensors", weights_path=wdir),
                    log=lambda *a: None)
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ROOT=ROOT, MODEL=model,
                   AKAP_MOE_MODE=moe_mode, WEIGHTS=wdir, PROMPTS=json.dumps(PROMPTS))
        procs.append(subprocess.Popen([sys.executable, "-c", CHILD], env=env, cwd=ROOT,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-3000:] for o in outs]
    tp_out = json.loads([l for l in outs[0][0].splitlines() if l.startswith("RESULT ")][0][7:])
    # every TP token is (near-)argmax of the dense reference on the SOURCE weights
    for p, out in zip(PROMPTS, tp_out):
        logits = dense_logits(src, p + out).float()
        for i, tok in enumerate(out):
            row = logits[len(p) - 1 + i]
            gap = (row.max() - row[tok]).item() / (row.std().item() + 1e-6)
            assert gap <= 0.1, (i, tok, gap)
    one = ref.generate(None, SamplingParams(max_tokens=6, temperature=0, ignore_eos=True),
                       prompt_ids=PROMPTS)
    agree = sum(a == b for o, t in zip(one, tp_out) for a, b in zip(o.output_ids, t))
    assert agree >= 0.8 * sum(len(t) for t in tp_out)


def test_qwen3_moe_hf_config_and_names():
    """A Qwen3-MoE config.json maps to arch qwen3_moe (q/k norm, moe_intermediate_size as the
    expert FFN, num_experts, norm_topk_prob) and its experts load from mlp.experts.* names."""
    from aws_k8s_ansible_provisioner_amd.models.config import ModelConfig

    d = {"model_type": "qwen3_moe", "vocab_size": 151936, "hidden_size": 2048,
         "intermediate_size": 6144, "moe_intermediate_size": 768, "num_hidden_layers": 48,
         "num_attention_heads": 32, "num_key_value_heads": 4, "head_dim": 128,
         "num_experts": 128, "num_experts_per_tok": 8, "norm_topk_prob": True,
         "rope_theta": 1000000.0, "max_position_embeddings": 40960}
    c = ModelConfig.from_hf_dict("q", d)
    assert (c.arch, c.qk_norm, c.intermediate_size, c.num_experts, c.experts_per_token,
            c.moe_renormalize) == ("qwen3_moe", True, 768, 128, 8, True)
    from aws_k8s_ansible_provisioner_amd.models.config import get_config

    ref = get_config("qwen3-30b-a3b")
    for f in ("hidden_size", "intermediate_size", "num_layers", "num_heads", "num_kv_heads",
              "num_experts", "experts_per_token", "vocab_size"):
        assert getattr(ref, f) == getattr(c, f), f
    assert 30e9 < ref.num_params() < 31e9
