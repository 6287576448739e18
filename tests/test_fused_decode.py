"""Fused decode layer chain (4 dgemm launches per layer: residual add + next-norm elementwise
half in the O / down epilogues, norm row scale in the consumer epilogue, SwiGLU in the
gate|up epilogue) vs the regular decode forward of the same model and inputs.

CPU: the ops' torch reference paths (chain bookkeeping: sums of squares, residual stream,
norm weights per position).  GPU: the HIP kernels, split-K and prefetch variants included.
"""
import dataclasses

import pytest
import torch

from aws_k8s_ansible_provisioner_amd import ops
from aws_k8s_ansible_provisioner_amd.models.config import get_config
from aws_k8s_ansible_provisioner_amd.models.transformer import AttnBatch, DecoderLM


def _setup(name, device, B=8, ctx=40, bs=32, seed=0):
    cfg = get_config(name)
    torch.manual_seed(seed)
    m = DecoderLM(cfg, device=device, seed=seed, max_model_len=256, init_std=0.05)
    nblk = (ctx + bs) // bs + 1
    kv = m.allocate_kv_cache(B * nblk + 1, bs)
    kv.copy_((torch.randn(kv.shape, device=device) * 0.5).to(kv.dtype))
    ks, vs = m.cache_views(kv, bs)
    bt = torch.arange(B * nblk, dtype=torch.int32, device=device).view(B, nblk)
    seq_lens = torch.tensor([ctx - 3 * i for i in range(B)], dtype=torch.int32, device=device)
    pos = (seq_lens - 1).long()
    slots = bt.long().gather(1, (pos // bs).view(-1, 1)).view(-1) * bs + pos % bs
    batch = AttnBatch(False, pos, slots, bt, seq_lens,
                      torch.arange(B + 1, dtype=torch.int32, device=device))
    if device != "cpu":
        batch.workspace = ops.decode_workspace(B, m.hkv, m.hq // m.hkv, 1, device)
    ids = torch.randint(0, cfg.vocab_size, (B,), device=device)
    return m, batch, ids, ks, vs


def _compare(name, device, plan):
    m, batch, ids, ks, vs = _setup(name, device)
    base = m.forward(ids, batch, ks, vs).float()
    fused = m._forward_fused_decode(ids, batch, ks, vs, plan).float()
    err = (fused - base).abs().max().item()
    scale = base.abs().max().item()
    assert err <= 3e-2 * scale + 3e-2, f"max err {err:.4g} vs scale {scale:.4g}"
    lb = m.compute_logits(base.to(m.dtype)).float()
    lf = m.compute_logits(fused.to(m.dtype)).float()
    agree = (lb.argmax(-1) == lf.argmax(-1)).float().mean().item()
    assert agree >= 0.75, f"greedy agreement {agree}"


PLAIN_PLAN = {"w_qkv": (1, 1, 0), "w_o": (1, 1, 0), "w_gate_up": (1, 1, 0), "w_down": (1, 1, 0)}


@pytest.mark.parametrize("name", ["tiny-qwen3", "tiny-llama"])
def test_fused_decode_chain_cpu(name):
    _compare(name, "cpu", PLAIN_PLAN)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["tiny-qwen3", "tiny-llama"])
@pytest.mark.parametrize("plan", [
    PLAIN_PLAN,
    {"w_qkv": (1, 4, 0), "w_o": (2, 2, 0), "w_gate_up": (1, 2, 0), "w_down": (2, 2, 0)},
    {"w_qkv": (2, 2, 0), "w_o": (1, 4, 0), "w_gate_up": (1, 4, 0), "w_down": (1, 4, 0)},
    {"w_qkv": (1, 1, 128), "w_o": (1, 1, 64), "w_gate_up": (1, 1, 128), "w_down": (2, 1, 64)},
    # kgemm.hip (K split inside the workgroup) for the plain qkv and the residual epilogues
    {"w_qkv": (1, 1, 0, 0, False, 32), "w_o": (1, 1, 0, 0, False, 16), "w_gate_up": (1, 2, 0),
     "w_down": (1, 1, 0, 0, False, 32)},
])
def test_fused_decode_chain_gpu(name, plan):
    ops.load_native(required=True)
    _compare(name, "cuda", plan)


@pytest.mark.gpu
def test_fused_epilogues_gpu():
    """EPI_RESNORM (residual, a_out, sums of squares) and EPI_SILU against fp32 references."""
    ops.load_native(required=True)
    torch.manual_seed(5)
    dev = "cuda"
    for M, N, K, s in [(37, 1024, 2048, 1), (64, 1024, 2048, 4), (256, 512, 1024, 2)]:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.03
        res = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        res0 = res.clone()
        ln = torch.rand(N, device=dev, dtype=torch.bfloat16) + 0.5
        ss = torch.zeros(M, device=dev)
        ssi = torch.rand(M, device=dev) * K + 1.0
        a = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ops.dgemm(x, w, splitk=s, pf=2, out=res, epi=ops.EPI_RESNORM, ss_out=ss, a_out=a,
                  ln_out=ln, ss_in=ssi)
        y = (x.float() @ w.float().t()) * torch.rsqrt(ssi / K + 1e-6)[:, None]
        want = (y.to(torch.bfloat16).float() + res0.float())
        assert (res.float() - want).abs().max().item() <= 2e-2 * want.abs().max().item()
        assert (a.float() - res.float() * ln.float()).abs().max().item() <= \
            1e-2 * a.float().abs().max().item()
        ssw = res.float().pow(2).sum(-1)
        assert torch.allclose(ss, ssw, rtol=1e-3, atol=1e-2)
        # SwiGLU epilogue over [gate; up] rows
        w2 = torch.randn(2 * N, K, device=dev, dtype=torch.bfloat16) * 0.03
        act = ops.dgemm(x, w2, pf=2, epi=ops.EPI_SILU, ss_in=ssi)
        gu = ((x.float() @ w2.float().t()) * torch.rsqrt(ssi / K + 1e-6)[:, None])
        want2 = ops.reference.silu_and_mul(gu.to(torch.bfloat16)).float()
        assert act.shape == (M, N)
        assert (act.float() - want2).abs().max().item() <= 2e-2 * want2.abs().max().item()


def test_gemm_tune_cache_round_trip(tmp_path):
    """The persisted plan reloads only for the same model shapes / batch buckets / library."""
    from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner

    m = DecoderLM(get_config("tiny-llama"), device="cpu", seed=0, max_model_len=64)
    Ms = [16, 32]
    w = m.layers[0].w_qkv
    gemm_tuner._PLAN.clear()
    gemm_tuner._FUSED.clear()
    gemm_tuner._PLAN[(16,) + tuple(w.shape)] = ("dgemm", 1, 1, 128, 4, False, 0, 128)
    gemm_tuner._PLAN[(32,) + tuple(w.shape)] = ("wgemm",)
    gemm_tuner._FUSED[32] = {"w_qkv": (1, 4, 0, 0, False, 0, 64),
                             "w_o": (1, 1, 0, 0, False, 32, 64)}
    want_plan, want_fused = dict(gemm_tuner._PLAN), dict(gemm_tuner._FUSED)
    path = str(tmp_path / "tune.json")
    gemm_tuner.save_cache(path, m, Ms)
    gemm_tuner._PLAN.clear()
    gemm_tuner._FUSED.clear()
    assert not gemm_tuner.load_cache(path, m, [16, 32, 64])  # other buckets: retune
    assert not gemm_tuner._PLAN
    cfg = dataclasses.replace(get_config("tiny-llama"), intermediate_size=2 * get_config(
        "tiny-llama").intermediate_size)
    other = DecoderLM(cfg, device="cpu", seed=0, max_model_len=64)
    assert not gemm_tuner.load_cache(path, other, Ms)          # other shapes: retune
    assert gemm_tuner.load_cache(path, m, Ms)
    assert gemm_tuner._PLAN == want_plan and gemm_tuner._FUSED == want_fused
    assert gemm_tuner.lookup(32, *w.shape) == ("wgemm",)
    gemm_tuner._PLAN.clear()
    gemm_tuner._FUSED.clear()
    assert not gemm_tuner.load_cache(str(tmp_path / "missing.json"), m, Ms)
