"""Decoder-only transformer (Qwen3 / Llama-3 / Mixtral) on the gfx950 kernels.

MI355X-first structure (not a module-per-op port):
  * fused weights: one QKV projection [ (Hq+2Hkv)*D, d ] and one gate|up projection
    [2F, d] per layer, so each layer is 4 large hipBLASLt GEMMs + 5 hand-written kernels
    (fused add+RMSNorm x2, QK-norm+RoPE+KV-write, paged attention, SiLU*mul);
  * the residual stream is updated in place by the fused add+norm kernel;
  * tensor parallel: QKV / gate_up column-split by heads / ffn rows, O / down row-split
    with one RCCL all-reduce each, vocab-parallel embedding + LM head;
  * everything in forward() is allocation-stable and sync-free on the decode path, so
    the engine captures it in a hipGraph per batch-size bucket.
"""
from __future__ import annotations

import dataclasses
import math
import os
from typing import Optional

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import reference as ref
from ..parallel import comm
from ..parallel.state import ParallelState, get_state
from .config import ModelConfig
from .moe import MoEBlock

FUSED_DECODE = os.environ.get("AKAP_FUSED_DECODE", "1") != "0"
PREFETCH_WEIGHTS = os.environ.get("AKAP_PREFETCH_WEIGHTS", "0") == "1"
FUSED_GEMM = os.environ.get("AKAP_FUSED_GEMM", "1") != "0"
# prefill attention applies the q norm + RoPE itself from the QKV rows (AKAP_PREFILL_QPREP=0:
# the standalone pass writes every q row, the kernel reads q)
PREFILL_QPREP = os.environ.get("AKAP_PREFILL_QPREP", "1") != "0"


@dataclasses.dataclass
class AttnBatch:
    """Flattened batch description consumed by the attention kernels."""
    is_prefill: bool
    positions: torch.Tensor      # [T] int64
    slots: torch.Tensor          # [T] int64 (-1 = padding)
    block_tables: torch.Tensor   # [B, max_blocks] int32
    seq_lens: torch.Tensor       # [B] int32
    q_start: torch.Tensor        # [B+1] int32
    tile_seq: Optional[torch.Tensor] = None  # prefill tile map
    tile_row: Optional[torch.Tensor] = None
    num_parts: int = 1           # decode split-KV partitions
    part_size: int = 512
    workspace: Optional[tuple] = None
    tile_rows: int = 64          # q rows per prefill tile of the map (128: flash-style kernel)
    num_decode: int = 0          # mixed step: leading single-token decode rows [0, num_decode)
    # V tail (GPU, bf16 cache): per-layer [slots, Hkv, 8, D] partial-group buffers and the
    # per-token (= per decode row) tail slot; None = the plain V cache write path
    v_tails: Optional[list] = None
    tail_slot: Optional[torch.Tensor] = None


@dataclasses.dataclass
class LayerWeights:
    ln1: torch.Tensor
    ln2: torch.Tensor
    w_qkv: torch.Tensor
    w_o: torch.Tensor
    q_norm: Optional[torch.Tensor]
    k_norm: Optional[torch.Tensor]
    w_gate_up: Optional[torch.Tensor]
    w_down: Optional[torch.Tensor]
    moe: Optional[MoEBlock] = None


def _shard_rows(w: torch.Tensor, rank: int, size: int) -> torch.Tensor:
    n = w.shape[0] // size
    return w[rank * n:(rank + 1) * n]


def _shard_cols(w: torch.Tensor, rank: int, size: int) -> torch.Tensor:
    n = w.shape[1] // size
    return w[:, rank * n:(rank + 1) * n]


def ipc_safe_alloc_bytes(nbytes: int) -> int:
    """Bytes to allocate for an `nbytes` buffer that a peer process will hipIpc-open: the
    caching allocator's 2 MiB rounding, then, if bit 31 of the size is set (size mod 4 GiB >=
    2 GiB -- hipIpcOpenMemHandle of such an allocation hangs on the ROCm 7.0.2 runtime that
    PyTorch bundles), the next multiple of 4 GiB."""
    r = -(-int(nbytes) // (2 << 20)) * (2 << 20)
    if r & (1 << 31):
        r = ((r >> 32) + 1) << 32
    return r


def kv_segment_layers(L: int, per_layer: int, max_segment_bytes: int,
                      ipc_safe: bool = True) -> int:
    """Layers per KV segment: as many as fit `max_segment_bytes`; with ipc_safe, the count in
    [max/2, max] whose segments need the fewest ipc_safe_alloc_bytes padding bytes (ties: the
    fewest segments)."""
    lps_max = max(1, min(L, max_segment_bytes // max(1, per_layer)))
    if not ipc_safe:
        return lps_max

    def pad_total(lps: int) -> int:
        return sum(ipc_safe_alloc_bytes(min(lps, L - l0) * per_layer) -
                   min(lps, L - l0) * per_layer for l0 in range(0, L, lps))

    return min(range(lps_max, lps_max // 2, -1), key=pad_total)


class DecoderLM:
    """Weights + forward for one tensor-parallel rank."""

    def __init__(self, cfg: ModelConfig, device: torch.device | str = "cpu",
                 dtype: torch.dtype = torch.bfloat16, seed: int = 0,
                 pstate: Optional[ParallelState] = None, max_model_len: int = 4096,
                 full_then_shard: bool = False, init_std: float = 0.02):
        self.cfg = cfg
        self.init_std = init_std
        self.device = torch.device(device)
        self.dtype = dtype
        self.ps = pstate or get_state()
        tp, r = self.ps.tp_size, self.ps.tp_rank
        if cfg.num_heads % tp:
            raise ValueError("num_heads must divide by tp")
        self.hq = cfg.num_heads // tp
        self.hkv = max(1, cfg.num_kv_heads // tp)
        self.kv_replicas = max(1, tp // cfg.num_kv_heads)
        self.D = cfg.head_dim
        self.ffn = cfg.intermediate_size // tp
        self.vocab_per = math.ceil(cfg.vocab_size / tp)
        self.vocab_start = r * self.vocab_per
        self.vocab_end = min(cfg.vocab_size, self.vocab_start + self.vocab_per)
        self.scale = 1.0 / math.sqrt(self.D)
        if max_model_len > cfg.max_position:
            # the rotary table (and the kernels that index it by position) end there
            raise ValueError(f"max_model_len {max_model_len} exceeds {cfg.name}'s "
                             f"max_position_embeddings {cfg.max_position}")
        self._init_weights(seed, full_then_shard)
        self.cos_sin = ref.rope_cos_sin(min(cfg.max_position, max(max_model_len, 16)), self.D,
                                        cfg.rope_theta, cfg.rope_scaling, device=self.device)

    # ------------------------------------------------------------------ weights
    def _rand(self, g: torch.Generator, *shape, std: Optional[float] = None) -> torch.Tensor:
        t = torch.empty(*shape, dtype=torch.float32, device=g.device)
        t.normal_(0.0, self.init_std if std is None else std, generator=g)
        return t.to(self.dtype)

    def _init_weights(self, seed: int, full_then_shard: bool) -> None:
        cfg, tp, r = self.cfg, self.ps.tp_size, self.ps.tp_rank
        d, D = cfg.hidden_size, self.D
        gdev = self.device if self.device.type == "cuda" else torch.device("cpu")
        # Full-then-shard (tests): identical logical weights for any tp.  Otherwise each
        # rank draws only its shard (70B at TP=8 never materialises the full model).
        g = torch.Generator(device=gdev)
        g.manual_seed(seed if full_then_shard else seed * 1000 + r)
        to = dict(device=self.device)
        one = lambda n: torch.ones(n, dtype=self.dtype, **to)  # noqa: E731

        vp = self.vocab_per
        if full_then_shard:
            emb_full = self._rand(g, vp * tp, d)
            emb_full[cfg.vocab_size:] = 0
            self.embed = emb_full[r * vp:(r + 1) * vp].contiguous().to(**to)
        else:
            self.embed = self._rand(g, vp, d).to(**to)
            self.embed[self.vocab_end - self.vocab_start:] = 0
        self.layers: list[LayerWeights] = []
        for _ in range(cfg.num_layers):
            if full_then_shard:
                wq = self._rand(g, cfg.q_size, d)
                wk = self._rand(g, cfg.kv_size, d)
                wv = self._rand(g, cfg.kv_size, d)
                wo = self._rand(g, d, cfg.q_size)
                q_sh = _shard_rows(wq, r, tp)
                k0, k1 = self._kv_head_range()
                k_sh, v_sh = wk[k0 * D:k1 * D], wv[k0 * D:k1 * D]
                w_qkv = torch.cat([q_sh, k_sh, v_sh], 0).contiguous().to(**to)
                w_o = _shard_cols(wo, r, tp).contiguous().to(**to)
            else:
                w_qkv = self._rand(g, (self.hq + 2 * self.hkv) * D, d).to(**to)
                w_o = self._rand(g, d, self.hq * D).to(**to)
            qn = one(D) if cfg.qk_norm else None
            kn = one(D) if cfg.qk_norm else None
            if cfg.is_moe:
                moe = MoEBlock(cfg, self.ps, self.device, self.dtype, g, full_then_shard,
                               std=self.init_std)
                lw = LayerWeights(one(d), one(d), w_qkv, w_o, qn, kn, None, None, moe)
            else:
                if full_then_shard:
                    wg = self._rand(g, cfg.intermediate_size, d)
                    wu = self._rand(g, cfg.intermediate_size, d)
                    wd = self._rand(g, d, cfg.intermediate_size)
                    w_gu = torch.cat([_shard_rows(wg, r, tp), _shard_rows(wu, r, tp)], 0).contiguous().to(**to)
                    w_d = _shard_cols(wd, r, tp).contiguous().to(**to)
                else:
                    w_gu = self._rand(g, 2 * self.ffn, d).to(**to)
                    w_d = self._rand(g, d, self.ffn).to(**to)
                lw = LayerWeights(one(d), one(d), w_qkv, w_o, qn, kn, w_gu, w_d)
            self.layers.append(lw)
        self.final_norm = one(d)
        if cfg.tie_embeddings:
            self.lm_head = self.embed
        elif full_then_shard:
            lm = self._rand(g, vp * tp, d)
            lm[cfg.vocab_size:] = 0
            self.lm_head = lm[r * vp:(r + 1) * vp].contiguous().to(**to)
        else:
            self.lm_head = self._rand(g, vp, d).to(**to)
            self.lm_head[self.vocab_end - self.vocab_start:] = 0

    def _kv_head_range(self) -> tuple[int, int]:
        """kv heads owned by this TP rank (replicated when tp > num_kv_heads)."""
        tp, r, H = self.ps.tp_size, self.ps.tp_rank, self.cfg.num_kv_heads
        if H >= tp:
            return r * H // tp, (r + 1) * H // tp
        h = r // (tp // H)
        return h, h + 1

    @property
    def graph_safe(self) -> bool:
        """Decode step free of host syncs (capturable in a hipGraph)."""
        return all(l.moe is None or l.moe.graph_safe for l in self.layers)

    def weight_bytes(self) -> int:
        n = self.embed.numel() + self.final_norm.numel()
        if self.lm_head is not self.embed:
            n += self.lm_head.numel()
        for lw in self.layers:
            for t in (lw.ln1, lw.ln2, lw.w_qkv, lw.w_o, lw.q_norm, lw.k_norm, lw.w_gate_up,
                      lw.w_down):
                if t is not None:
                    n += t.numel()
            if lw.moe is not None:
                n += lw.moe.numel()
        return n * 2

    def hf_state_dict(self) -> dict:
        """This (unsharded, tp=1) model's weights under HF names, un-fusing QKV and gate|up
        and the Mixtral experts -- the inverse of load_state_dict (checkpoint export and the
        loader's round-trip tests)."""
        if self.ps.tp_size != 1:
            raise ValueError("hf_state_dict needs the unsharded (tp=1) model")
        cfg, D = self.cfg, self.D
        n = self.vocab_end - self.vocab_start
        sd = {"model.embed_tokens.weight": self.embed[:n].clone(),
              "model.norm.weight": self.final_norm.clone()}
        if not cfg.tie_embeddings:
            sd["lm_head.weight"] = self.lm_head[:n].clone()
        q, kv = self.hq * D, self.hkv * D
        for i, lw in enumerate(self.layers):
            p = f"model.layers.{i}."
            sd[p + "input_layernorm.weight"] = lw.ln1.clone()
            sd[p + "post_attention_layernorm.weight"] = lw.ln2.clone()
            sd[p + "self_attn.q_proj.weight"] = lw.w_qkv[:q].clone()
            sd[p + "self_attn.k_proj.weight"] = lw.w_qkv[q:q + kv].clone()
            sd[p + "self_attn.v_proj.weight"] = lw.w_qkv[q + kv:].clone()
            sd[p + "self_attn.o_proj.weight"] = lw.w_o.clone()
            if lw.q_norm is not None:
                sd[p + "self_attn.q_norm.weight"] = lw.q_norm.clone()
                sd[p + "self_attn.k_norm.weight"] = lw.k_norm.clone()
            if lw.moe is not None:
                sd.update(lw.moe.hf_state_dict(p))
            else:
                F_ = lw.w_gate_up.shape[0] // 2
                sd[p + "mlp.gate_proj.weight"] = lw.w_gate_up[:F_].clone()
                sd[p + "mlp.up_proj.weight"] = lw.w_gate_up[F_:].clone()
                sd[p + "mlp.down_proj.weight"] = lw.w_down.clone()
        return sd

    def load_state_dict(self, sd: dict) -> None:
        """Load HF-named tensors (safetensors from the model PVC) into the fused layout."""
        cfg, tp, r = self.cfg, self.ps.tp_size, self.ps.tp_rank
        cp = lambda dst, src: dst.copy_(src.to(dst.dtype))  # noqa: E731
        emb = sd["model.embed_tokens.weight"]
        n = self.vocab_end - self.vocab_start
        cp(self.embed[:n], emb[self.vocab_start:self.vocab_end])
        for i, lw in enumerate(self.layers):
            p = f"model.layers.{i}."
            cp(lw.ln1, sd[p + "input_layernorm.weight"])
            cp(lw.ln2, sd[p + "post_attention_layernorm.weight"])
            q = _shard_rows(sd[p + "self_attn.q_proj.weight"], r, tp)
            k0, k1 = self._kv_head_range()
            D = self.D
            k = sd[p + "self_attn.k_proj.weight"][k0 * D:k1 * D]
            v = sd[p + "self_attn.v_proj.weight"][k0 * D:k1 * D]
            cp(lw.w_qkv, torch.cat([q, k, v], 0))
            cp(lw.w_o, _shard_cols(sd[p + "self_attn.o_proj.weight"], r, tp))
            if lw.q_norm is not None:
                cp(lw.q_norm, sd[p + "self_attn.q_norm.weight"])
                cp(lw.k_norm, sd[p + "self_attn.k_norm.weight"])
            if lw.moe is not None:
                lw.moe.load_state_dict(sd, p)
            else:
                g_ = _shard_rows(sd[p + "mlp.gate_proj.weight"], r, tp)
                u_ = _shard_rows(sd[p + "mlp.up_proj.weight"], r, tp)
                cp(lw.w_gate_up, torch.cat([g_, u_], 0))
                cp(lw.w_down, _shard_cols(sd[p + "mlp.down_proj.weight"], r, tp))
        cp(self.final_norm, sd["model.norm.weight"])
        if not cfg.tie_embeddings:
            cp(self.lm_head[:n], sd["lm_head.weight"][self.vocab_start:self.vocab_end])

    # ------------------------------------------------------------------ kv cache
    def allocate_kv_cache(self, num_blocks: int, block_size: int,
                          kv_dtype: str = "auto") -> torch.Tensor:
        """The whole cache as ONE allocation [L, 2, NB, Hkv*BS*D] (micro-benchmarks, tests)."""
        return self.allocate_kv_segments(num_blocks, block_size, kv_dtype,
                                         max_segment_bytes=1 << 62)[0]

    def allocate_kv_segments(self, num_blocks: int, block_size: int, kv_dtype: str = "auto",
                             max_segment_bytes: Optional[int] = None) -> list:
        """Layer-range segments [Ls, 2, NB, Hkv*BS*D] (K block = [Hkv,BS,D], V block =
        [Hkv,BS/8,D,8]) of at most `max_segment_bytes` each (AKAP_KV_SEGMENT_GIB, default 32),
        zero-filled so never-written slots read as finite zeros.  kv_dtype "fp8": uint8
        storage of OCP e4m3fn values (half the bytes of bf16).  Each segment is its own
        allocation, exported by hipIpc on its own (P/D pull).

        On the GPU every allocation's size is kept hipIpc-safe (`ipc_safe_alloc_bytes`): the
        HIP runtime PyTorch bundles (ROCm 7.0.2) hangs in hipIpcOpenMemHandle when bit 31 of
        the allocation size is set (size mod 4 GiB >= 2 GiB; 1.5 / 5 / 8 / 9.5 / 36 GiB map,
        2 / 2.5 / 6.6 GiB hang, at any occupancy -- bench/ipc_import_repro.cpp,
        profiles/r6_ipc_import_sweep.md; ROCm 7.2's runtime maps them all).  That was the
        round-4/5 "hang once the device is mostly allocated": big caches made such sizes.
        The layers per segment are chosen to avoid padding where possible; otherwise the
        allocation is padded to the next 4 GiB multiple (the tail is never addressed)."""
        per_block = self.hkv * block_size * self.D
        dt = torch.uint8 if kv_dtype.startswith("fp8") else self.dtype
        if max_segment_bytes is None:
            max_segment_bytes = int(float(os.environ.get("AKAP_KV_SEGMENT_GIB", "32")) * 2**30)
        L = self.cfg.num_layers
        es = torch.empty(0, dtype=dt).element_size()
        per_layer = 2 * num_blocks * per_block * es
        gpu = torch.device(self.device).type == "cuda"
        lps = kv_segment_layers(L, per_layer, max_segment_bytes, ipc_safe=gpu)
        segs = []
        for l0 in range(0, L, lps):
            n = min(lps, L - l0)
            elems = n * 2 * num_blocks * per_block
            alloc = ipc_safe_alloc_bytes(elems * es) // es if gpu else elems
            buf = torch.zeros(alloc, dtype=dt, device=self.device)
            segs.append(buf[:elems].view(n, 2, num_blocks, per_block))
        return segs

    def cache_views(self, kv, block_size: int):
        """Per-layer K / V views of the cache (one tensor or its list of layer segments)."""
        segs = list(kv) if isinstance(kv, (list, tuple)) else [kv]
        ks, vs = [], []
        for seg in segs:
            NB = seg.shape[2]
            ks += [seg[l, 0].view(NB, self.hkv, block_size, self.D) for l in range(seg.shape[0])]
            vs += [seg[l, 1].view(NB, self.hkv, block_size // 8, self.D, 8)
                   for l in range(seg.shape[0])]
        return ks, vs

    # ------------------------------------------------------------------ forward
    def embed_tokens(self, ids: torch.Tensor) -> torch.Tensor:
        x = ops.embedding(ids, self.embed, vocab_start=self.vocab_start, vocab_end=self.vocab_end)
        return comm.tp_all_reduce(x)

    def _attention(self, q, batch: AttnBatch, kc, vc, out, vt=None, qprep=None):
        if batch.is_prefill:
            nd = batch.num_decode
            if nd and q.is_cuda:
                # mixed step: the decode rows lead the batch and run the split-KV decode
                # kernel; the prefill tile map covers only the prefill rows after them
                # (on CPU the reference attention handles every row at once)
                ops.paged_attention_decode(out[:nd], q[:nd], kc, vc, batch.block_tables[:nd],
                                           batch.seq_lens[:nd], self.hq // self.hkv,
                                           self.scale, workspace=batch.workspace,
                                           num_parts=batch.num_parts,
                                           part_size=batch.part_size, v_tail=vt,
                                           tail_slot=batch.tail_slot)
            ops.paged_attention_prefill(out, q, kc, vc, batch.block_tables, batch.seq_lens,
                                        batch.q_start, batch.tile_seq, batch.tile_row,
                                        self.hq // self.hkv, self.scale,
                                        tile_rows=batch.tile_rows, qprep=qprep)
        else:
            ops.paged_attention_decode(out, q, kc, vc, batch.block_tables, batch.seq_lens,
                                       self.hq // self.hkv, self.scale, workspace=batch.workspace,
                                       num_parts=batch.num_parts, part_size=batch.part_size,
                                       v_tail=vt, tail_slot=batch.tail_slot)
        return out

    def forward(self, input_ids: torch.Tensor, batch: AttnBatch, k_caches, v_caches
                ) -> torch.Tensor:
        cfg = self.cfg
        T = input_ids.shape[0]
        eps = cfg.rms_eps
        if (not batch.is_prefill and FUSED_DECODE and FUSED_GEMM and self.device.type == "cuda"
                and all(l.moe is None for l in self.layers)):
            from ..ops import gemm_tuner

            plan = gemm_tuner.fused_plan(T)
            if plan is not None:
                return self._forward_fused_decode(input_ids, batch, k_caches, v_caches, plan)
        x = self.embed_tokens(input_ids)
        residual = x
        h = ops.rms_norm(x, self.layers[0].ln1, eps)
        x = None
        for li, lw in enumerate(self.layers):
            if li > 0:
                h, residual = ops.fused_add_rms_norm(x, residual, lw.ln1, eps)
            qkv = ops.linear(h, lw.w_qkv)
            attn = torch.empty(T, self.hq, self.D, dtype=self.dtype, device=self.device)
            if not batch.is_prefill and PREFETCH_WEIGHTS:
                # warm this layer's remaining GEMM weights (+ the next QKV) in MALL before
                # the HBM-bound attention stream; the latency-bound GEMMs then hit cache
                nxt = self.layers[li + 1].w_qkv if li + 1 < len(self.layers) else None
                ops.l2_prefetch([lw.w_o, lw.w_gate_up, lw.w_down, nxt])
            vt = batch.v_tails[li] if batch.v_tails is not None else None
            if not batch.is_prefill and FUSED_DECODE:
                # q/k-norm + RoPE + KV-cache write fused into the decode attention kernel
                ops.paged_attention_decode_fused(
                    attn, qkv, k_caches[li], v_caches[li], batch.block_tables, batch.seq_lens,
                    batch.positions, batch.slots, self.cos_sin, lw.q_norm, lw.k_norm,
                    self.hq // self.hkv, self.scale, eps, workspace=batch.workspace,
                    num_parts=batch.num_parts, part_size=batch.part_size, v_tail=vt,
                    tail_slot=batch.tail_slot)
            else:
                q = torch.empty_like(attn)
                # prefill on the GPU: the attention kernel norms + rotates its own q rows from
                # the QKV projection, so the standalone pass writes q only for the decode rows
                qp = batch.is_prefill and PREFILL_QPREP and qkv.is_cuda
                ops.qk_norm_rope_cache(qkv, q, k_caches[li], v_caches[li], batch.positions,
                                       batch.slots, self.cos_sin, lw.q_norm, lw.k_norm, self.hq,
                                       self.hkv, eps, True, decode=not batch.is_prefill,
                                       v_tail=vt, tail_slot=batch.tail_slot,
                                       num_decode=batch.num_decode if batch.is_prefill else 0,
                                       q_rows=batch.num_decode if qp else -1)
                self._attention(q, batch, k_caches[li], v_caches[li], attn, vt,
                                qprep=(qkv, batch.positions, self.cos_sin, lw.q_norm, eps)
                                if qp else None)
            o = comm.tp_all_reduce(ops.linear(attn.view(T, self.hq * self.D), lw.w_o))
            h, residual = ops.fused_add_rms_norm(o, residual, lw.ln2, eps)
            if lw.moe is not None:
                x = lw.moe.forward(h)
            else:
                x = comm.tp_all_reduce(ops.linear(ops.linear_silu(h, lw.w_gate_up), lw.w_down))
        h, _ = ops.fused_add_rms_norm(x, residual, self.final_norm, eps)
        return h

    def _forward_fused_decode(self, input_ids, batch: AttnBatch, k_caches, v_caches, plan: dict
                              ) -> torch.Tensor:
        """Dense decode step as 4 fused GEMM launches + 1 attention launch per layer
        (csrc/kernels/dgemm.hip): the residual add and the elementwise half of the next
        RMSNorm run in the O / down projections' epilogues (which also accumulate the
        per-row sum of squares), the norm's row scale in the consumer GEMM's epilogue, and
        SwiGLU in the gate|up projection's epilogue -- no separate norm / activation kernels.
        Tensor parallel: the row-parallel O / down projections store their partial sums and
        the residual epilogue moves into the all-reduce (comm.tp_all_reduce_resnorm: the
        custom xGMI kernel applies it in its store pass), so a TP layer is still 4 GEMM
        launches + 2 all-reduce launches + attention.  Plan from gemm_tuner.tune_fused:
        projection -> (split-K, prefetch depth, LDS-DMA tile width[, ring, in-launch])."""
        from ..ops import gemm_tuner

        T = input_ids.shape[0]
        eps = self.cfg.rms_eps
        L = len(self.layers)

        def cfg_(name):  # plan entry (split-K, prefetch, tile width[, ring, in-launch combine,
            #                            kgemm rows])
            e = tuple(plan[name])
            s_, p_ = e[:2]
            b_, n_, i_, k_, m_ = gemm_tuner.variant_fields(e[2:])[:5]
            return dict(splitk=s_, pf=p_, bn=b_, ns=n_, inlaunch=bool(i_), km=k_, bm=m_)

        c_qkv, c_o, c_gu, c_d = (cfg_(n) for n in ("w_qkv", "w_o", "w_gate_up", "w_down"))
        tp = self.ps.tp_size
        if tp == 1:
            # one launch (ops.embedding_prep): the embedding rows, the first layer's
            # un-normalised input and its row sums of squares (the first projection applies
            # the rsqrt, like every later one), and the zeroed per-layer accumulators
            ssb = torch.empty(2 * L + 1, T, dtype=torch.float32, device=self.device)
            ss, ss_in = ssb[:2 * L], ssb[2 * L]
            residual = torch.empty(T, self.cfg.hidden_size, dtype=self.dtype, device=self.device)
            a1 = torch.empty_like(residual)
            ops.embedding_prep(input_ids, self.embed, self.layers[0].ln1, residual, a1, ss_in,
                               ss, self.vocab_start, self.vocab_end)
        else:
            residual = self.embed_tokens(input_ids)
            ss = torch.zeros(2 * L, T, dtype=torch.float32, device=self.device)
            a1 = ops.rms_norm(residual, self.layers[0].ln1, eps)
            ss_in = None
        for li, lw in enumerate(self.layers):
            nxt = self.layers[li + 1].w_qkv if li + 1 < L else None
            qkv = ops.dgemm(a1, lw.w_qkv, eps=eps, ss_in=ss_in, **c_qkv)
            attn = torch.empty(T, self.hq, self.D, dtype=self.dtype, device=self.device)
            if PREFETCH_WEIGHTS:  # A/B knob: warm the layer's remaining weights in MALL
                ops.l2_prefetch([lw.w_o, lw.w_gate_up, lw.w_down, nxt])
            ops.paged_attention_decode_fused(
                attn, qkv, k_caches[li], v_caches[li], batch.block_tables, batch.seq_lens,
                batch.positions, batch.slots, self.cos_sin, lw.q_norm, lw.k_norm,
                self.hq // self.hkv, self.scale, eps, workspace=batch.workspace,
                num_parts=batch.num_parts, part_size=batch.part_size,
                v_tail=batch.v_tails[li] if batch.v_tails is not None else None,
                tail_slot=batch.tail_slot)
            a2 = torch.empty_like(residual)
            if tp > 1:
                part = ops.dgemm(attn.view(T, self.hq * self.D), lw.w_o, eps=eps, **c_o)
                comm.tp_all_reduce_resnorm(part, residual, lw.ln2, a2, ss[2 * li])
            else:
                ops.dgemm(attn.view(T, self.hq * self.D), lw.w_o, eps=eps, out=residual,
                          epi=ops.EPI_RESNORM, ss_out=ss[2 * li], a_out=a2, ln_out=lw.ln2,
                          **c_o)
            act = ops.dgemm(a2, lw.w_gate_up, eps=eps, ss_in=ss[2 * li], epi=ops.EPI_SILU,
                            **c_gu)
            if li + 1 < L:
                a1 = torch.empty_like(residual)
                if tp > 1:
                    part = ops.dgemm(act, lw.w_down, eps=eps, **c_d)
                    comm.tp_all_reduce_resnorm(part, residual, self.layers[li + 1].ln1, a1,
                                               ss[2 * li + 1])
                else:
                    ops.dgemm(act, lw.w_down, eps=eps, out=residual, epi=ops.EPI_RESNORM,
                              ss_out=ss[2 * li + 1], a_out=a1, ln_out=self.layers[li + 1].ln1,
                              **c_d)
                ss_in = ss[2 * li + 1]
            else:
                x = comm.tp_all_reduce(ops.dgemm(act, lw.w_down, eps=eps, **c_d))
        h, _ = ops.fused_add_rms_norm(x, residual, self.final_norm, eps)
        return h

    def compute_logits(self, h: torch.Tensor) -> torch.Tensor:
        logits = ops.linear(h, self.lm_head)
        if self.ps.tp_size > 1:
            logits = comm.tp_all_gather_last(logits)
        return logits[:, : self.cfg.vocab_size]
