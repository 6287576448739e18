"""Model runner: weights, the paged KV cache, device batch buffers and hipGraph decode.

* KV cache: ONE allocation [L, 2, NB, Hkv*BS*D] sized from the HBM left after weights
  (288 GB per MI355X -> millions of cached tokens for small models), zero-filled.
* Host->device: the C++ scheduler writes the batch into pinned host buffers; the runner
  issues a handful of non-blocking H2D copies into persistent device buffers.
* Decode: the whole step -- embedding, 28+ layers, LM head, fp32 cast, sampler -- is
  captured once per batch-size bucket into a hipGraph (torch.cuda.CUDAGraph is hipGraph
  on ROCm) and replayed with padded rows (seq_len 0, slot -1 => no work, no cache write).
* Prefill / chunked prefill: eager, variable T, tile-mapped MFMA attention.
"""
from __future__ import annotations

import math
import os
import time
from typing import Optional

import numpy as np
import torch

from ..utils import profiling
from .. import ops
from ..models import moe as moe_mod
from ..models.config import ModelConfig
from ..models.transformer import AttnBatch, DecoderLM
from ..parallel.state import ParallelState, drain_pending_collectives, get_state
from .config import EngineConfig

# decode staging H2D as a kernel reading the pinned buffer (1) or hipMemcpyAsync (0, A/B)
H2D_KERNEL = os.environ.get("AKAP_H2D_KERNEL", "1") != "0"

DEFAULT_BUCKETS = [1, 2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320,
                   384, 448, 512]


# per-step decode inputs (one row per sequence), staged together: see _stage_decode
DECODE_FIELDS = ("input_ids", "positions", "slots", "seeds", "seq_lens", "temperature", "top_p",
                 "top_k", "steps", "src_rows", "tail_slot")


# fault injection (tests/test_tp_gpu.py): a TP follower that skips its N-th decode replay, so
# its peers' custom collectives time out inside a replayed graph
_FAULT_SKIP_REPLAY = int(os.environ.get("AKAP_FAULT_SKIP_REPLAY", "0"))

class ModelRunner:
    def __init__(self, ecfg: EngineConfig, mcfg: ModelConfig,
                 pstate: Optional[ParallelState] = None, log=print):
        self.ecfg, self.mcfg = ecfg, mcfg
        self.ps = pstate or get_state()
        self.log = log
        dev = ecfg.resolved_device()
        if dev == "cuda":
            self.device = torch.device("cuda", torch.cuda.current_device())
            ops.load_native(required=True)  # GPU path never falls back to eager PyTorch
        else:
            self.device = torch.device("cpu")
        self.is_gpu = self.device.type == "cuda"
        t0 = time.time()
        self.model = DecoderLM(mcfg, self.device, seed=ecfg.seed, pstate=self.ps,
                               max_model_len=ecfg.max_model_len, init_std=ecfg.init_std,
                               full_then_shard=ecfg.shard_init == "full")
        if ecfg.load_format == "safetensors" and ecfg.weights_path:
            from .weights import load_safetensors_dir

            self.model.load_state_dict(load_safetensors_dir(ecfg.weights_path))
        self.log(f"[runner] model {mcfg.name} ready in {time.time() - t0:.1f}s "
                 f"({self.model.weight_bytes() / 2**30:.2f} GiB weights/rank)")
        self.bs = ecfg.block_size
        self.max_blocks = math.ceil(ecfg.max_model_len / self.bs)
        self.G = self.model.hq // self.model.hkv
        self.max_seqs = ecfg.max_num_seqs
        # a mixed step holds a full prefill token budget plus one decode row per sequence
        self.cap_tokens = ecfg.max_num_batched_tokens + self.max_seqs
        # prefill tile map granularity (flattened q rows per workgroup of the flash-style GPU
        # kernel; the CPU reference attention ignores the map): with the longest-first flat
        # grid (round 6) the 8-wave 256-row tile wins on long chunks (Qwen3 4 x 4096: 284.5 vs
        # 301.6 us, Llama-3-8B 32 x 512: 149.2 vs 154.5, 4 x 4096: 566.3 vs 578.8, q prep in
        # the kernel), the 128-row tile on chunks whose every prompt has <= 1024 rows (Qwen3
        # 32 x 512: 83.8 vs 87.9 us) -- profiles/r6_prefill_tile_order.md.  The 256-row kernel
        # needs a bf16 KV cache.
        bf16_kv = dev == "cuda" and not ecfg.kv_cache_dtype.startswith("fp8")
        self.tile_rows = 256 if bf16_kv else (128 if dev == "cuda" else 64)
        self.tile_rows_short = 128 if bf16_kv else 0
        if dev == "cuda" and os.environ.get("AKAP_PREFILL_TILE_ROWS") in ("128", "256"):
            self.tile_rows = int(os.environ["AKAP_PREFILL_TILE_ROWS"])  # A/B knob
            self.tile_rows_short = 0
            if self.tile_rows == 256 and ecfg.kv_cache_dtype.startswith("fp8"):
                self.tile_rows = 128  # the 256-row kernel needs a bf16 KV cache
        self.cap_tiles = self.cap_tokens * self.G // 64 + self.max_seqs + 1
        self.num_blocks = ecfg.num_gpu_blocks or self._derive_num_blocks()
        if self.ps.tp_size > 1:  # every TP rank must address the same block pool
            import torch.distributed as dist

            t = torch.tensor([self.num_blocks], dtype=torch.int64,
                             device=self.device if self.is_gpu else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.ps.tp_group)
            self.num_blocks = int(t.item())
        # layer-range segments, one allocation each (DecoderLM.allocate_kv_segments); `kv` is the
        # single tensor when one segment holds every layer (small caches, tests)
        self.kv_segs = self.model.allocate_kv_segments(self.num_blocks, self.bs,
                                                       ecfg.kv_cache_dtype)
        self.kv = self.kv_segs[0] if len(self.kv_segs) == 1 else None
        self.kv_dtype = self.kv_segs[0].dtype
        self.k_caches, self.v_caches = self.model.cache_views(self.kv_segs, self.bs)
        gib = sum(t.numel() * t.element_size() for t in self.kv_segs) / 2**30
        self.log(f"[runner] KV cache: {self.num_blocks} blocks x {self.bs} tokens "
                 f"({gib:.1f} GiB in {len(self.kv_segs)} allocation(s), "
                 f"{'fp8 e4m3' if self.kv_dtype == torch.uint8 else 'bf16'})")
        # V tail (see AttnParams.v_tail): one slot per live sequence (2x max_num_seqs, as P/D
        # activations can briefly exceed it; a sequence without a slot uses the plain path)
        self.v_tails: Optional[list] = None
        self.num_tail_slots = 0
        if self.v_tail_enabled():
            self.num_tail_slots = 2 * self.max_seqs
            self._tail = torch.zeros(mcfg.num_layers, self.num_tail_slots, self.model.hkv, 8,
                                     self.model.D, dtype=torch.bfloat16, device=self.device)
            self.v_tails = list(self._tail.unbind(0))
        # workspace sized for the finest split any bucket uses (256-token partitions)
        self.num_parts = max(1, math.ceil(ecfg.max_model_len / 128))
        self._alloc_buffers()
        self._hpre: Optional[torch.Tensor] = None  # prefill staging (pinned) + device mirror
        self._dpre: Optional[torch.Tensor] = None
        self.last_logprobs: Optional[np.ndarray] = None
        # top-N alternatives of the last step's sampled rows: (token ids [n, N], log-probs)
        self.last_top: Optional[tuple] = None
        self.graphs: dict[int, torch.cuda.CUDAGraph] = {}
        # decode graphs whose sampler also runs the top-k / top-p threshold passes: captured on
        # first use by a batch that needs them (single-rank engines; multi-rank engines capture
        # their only graphs with the passes, since a lazy capture would issue collectives alone)
        # decode graph variants by sampler mode (see _sample_mode), captured with the buckets
        self.graphs_v: dict[tuple, torch.cuda.CUDAGraph] = {}
        self._capture_mode: Optional[str] = None
        self.ep_overflow_steps = 0  # steps re-run after an EP dispatch overflow
        self.graph_pool = None
        self.buckets: list[int] = []
        if self.is_gpu and not ecfg.enforce_eager and self.model.graph_safe:
            self.capture_graphs()

    def v_tail_enabled(self) -> bool:
        """Decode keeps each sequence's partial 8-token V group in a token-major tail and
        writes the cache only in whole groups (csrc/kernels/attention.hip): GPU, bf16 KV
        cache, fused decode attention.  AKAP_V_TAIL=0 restores the per-token cache write."""
        from ..models import transformer as tfm

        return (self.is_gpu and self.kv_dtype == torch.bfloat16 and tfm.FUSED_DECODE and
                os.environ.get("AKAP_V_TAIL", "1") != "0" and
                not (self.ecfg.kv_role == "decode" and self.ps.tp_size > 1))

    def fill_tail(self, slot: int, block_table: list, n: int) -> None:
        """A sequence whose KV arrived whole (P/D decode side): copy its partial last V group
        (tokens [n & ~7, n)) from the cache into its tail before its first decode step."""
        if self.v_tails is None or slot < 0 or n % 8 == 0:
            return
        g0, cnt = n & ~7, n % 8
        blk, grp = int(block_table[g0 // self.bs]), (g0 % self.bs) // 8
        if self.is_gpu:
            # one launch for every layer (the tail-only form of the IPC pull kernel, reading
            # this engine's own cache) instead of a per-layer copy loop
            planes = self.kv_planes()
            ops.kv_pull(ops.plane_table(planes), self.num_blocks, planes, [], self.model.hkv,
                        self.bs, self.model.D, tail=self._tail, tail_jobs=[(blk, grp, cnt, slot)])
            return
        for vt, vc in zip(self.v_tails, self.v_caches):
            vt[slot, :, :cnt].copy_(vc[blk, :, grp, :, :cnt].transpose(-1, -2))

    def kv_planes(self) -> list:
        """The KV cache as [2 Ls planes, NB, block_elems] views, one per segment (bf16 views:
        fp8 bytes move in pairs)."""
        out = []
        for seg in self.kv_segs:
            kv = seg.view(torch.bfloat16) if seg.dtype == torch.uint8 else seg
            L, two, NB, be = kv.shape
            out.append(kv.view(L * two, NB, be))
        return out

    # ------------------------------------------------------------------ sizing
    def _derive_num_blocks(self) -> int:
        elem = 1 if self.ecfg.kv_cache_dtype.startswith("fp8") else 2
        per_block = self.mcfg.num_layers * 2 * self.model.hkv * self.bs * self.model.D * elem
        if not self.is_gpu:
            return max(64, min(4096, (self.max_seqs * self.ecfg.max_model_len) // self.bs + 8))
        torch.cuda.synchronize()
        free, total = torch.cuda.mem_get_info(self.device)
        # this process's own footprint (allocator + ~1 GiB of runtime / library state), not
        # the device-wide total - free: ranks that share one GPU (P/D or TP rehearsals) each
        # get their gpu_memory_utilization share, whichever sizes its cache first
        used = torch.cuda.memory_reserved(self.device) + 2**30
        d = self.mcfg.hidden_size
        width = d * 4 + (self.model.hq + 2 * self.model.hkv) * self.model.D + 3 * self.model.ffn
        act = self.cap_tokens * width * 2 * 3 + self.max_seqs * self.mcfg.vocab_size * 12
        reserve = act + 3 * 2**30
        budget = min(total * self.ecfg.gpu_memory_utilization - used, free) - reserve
        n = int(budget // per_block)
        if self.ecfg.kv_cache_max_gib:
            n = min(n, int(self.ecfg.kv_cache_max_gib * 2**30 // per_block))
        if n < self.max_blocks:
            raise RuntimeError(f"not enough HBM for the KV cache ({budget / 2**30:.1f} GiB)")
        return n

    def _pinned(self, n, dtype):
        t = torch.zeros(n, dtype=dtype, pin_memory=self.is_gpu)
        return t

    def _alloc_buffers(self) -> None:
        S, T, TL, mb = self.max_seqs, self.cap_tokens, self.cap_tiles, self.max_blocks
        spec = {
            "input_ids": (T, torch.int64), "positions": (T, torch.int64), "slots": (T, torch.int64),
            "seq_lens": (S, torch.int32), "q_start": (S + 1, torch.int32),
            "block_tables": (S * mb, torch.int32), "tile_seq": (TL, torch.int32),
            "tile_row": (TL, torch.int32), "logits_idx": (S, torch.int64),
            "req_ids": (S, torch.int64), "sample_mask": (S, torch.int32),
            "temperature": (S, torch.float32), "top_p": (S, torch.float32),
            "top_k": (S, torch.int32), "seeds": (S, torch.int64), "steps": (S, torch.int32),
            # decode lookahead: in-flight row whose sampled token is this row's input
            "src_rows": (S, torch.int64),
            # per token: its sequence's V-tail slot (-1: none)
            "tail_slot": (T, torch.int32),
        }
        self.h = {k: self._pinned(n, dt) for k, (n, dt) in spec.items()}
        self.np = {k: v.numpy() for k, v in self.h.items()}
        self.d = {k: torch.zeros(n, dtype=dt, device=self.device) for k, (n, dt) in spec.items()
                  if k not in ("req_ids", "sample_mask")}
        self.d_bt = self.d["block_tables"].view(S, mb)
        # decode staging: every per-step decode input packed in ONE pinned region and copied
        # to its device mirror by ONE H2D copy (instead of ten small copies, each a ~3 us
        # blit kernel plus a host launch, serialised ahead of the graph replay)
        fields = [(k, self.h[k].dtype, S) for k in DECODE_FIELDS] + [("block_tables", torch.int32,
                                                                      S * mb)]
        off, lay = 0, {}
        for k, dt, n in fields:
            lay[k] = (off, dt, n)
            off += -(-n * torch.empty(0, dtype=dt).element_size() // 16) * 16
        # two pinned staging regions used alternately: with a lookahead step in flight the
        # host stages step N+2 while step N+1's copy may still be queued behind step N
        self.hdecs = [self._pinned(off, torch.uint8) for _ in range(2)]
        self.ddec = torch.zeros(off, dtype=torch.uint8, device=self.device)
        view = lambda buf, o, dt, n: buf[o:o + n * torch.empty(0, dtype=dt).element_size()].view(dt)  # noqa: E731
        self.hd_nps = [{k: view(h, o, dt, n).numpy() for k, (o, dt, n) in lay.items()}
                       for h in self.hdecs]
        self._dslot = 0
        self.dd = {k: view(self.ddec, o, dt, n) for k, (o, dt, n) in lay.items()}
        # the staging kernel needs the pinned buffers' device mapping: probe it once, fall back
        # to hipMemcpyAsync where the host allocator does not provide one
        self._h2d_kernel = False
        if self.is_gpu and H2D_KERNEL:
            try:
                torch.ops.akap.h2d_stage(self.ddec[:16], self.hdecs[0][:16])
                self._h2d_kernel = True
            except RuntimeError as e:
                self.log(f"[runner] staging kernel unavailable ({e}); using hipMemcpyAsync")
        self.dd_bt = self.dd["block_tables"].view(S, mb)
        self._dec_bt_off = lay["block_tables"][0]
        self.out_tokens = torch.zeros(S, dtype=torch.int64, device=self.device)
        # sampled tokens of launched decode steps land here (one region per staging slot)
        self.tok_host = [self._pinned(S, torch.int64) for _ in range(2)]
        # error-word probes: slots 0/1 follow tok_host (lookahead), 2 the synchronous path,
        # 3..6 a TP follower's un-waited replays (_err_probe)
        self._err_host = [self._pinned(1, torch.int32) for _ in range(7)]
        self._pending_err = None
        self._follower_err: list = []
        self._follower_slot = 0
        self._replays = 0
        self.out_logprobs = torch.zeros(S, dtype=torch.float32, device=self.device)
        self.workspace = ops.decode_workspace(S, self.model.hkv, self.G, self.num_parts,
                                              self.device)

    def host_buffers(self) -> dict:
        return self.np

    def _stage_decode(self, n: int) -> int:
        """Host buffers (rows [0, n)) -> decode staging region -> device, one copy.  Returns
        the staging slot used (alternating)."""
        slot = self._dslot
        self._dslot ^= 1
        hd_np = self.hd_nps[slot]
        for k in DECODE_FIELDS:
            hd_np[k][:n] = self.np[k][:n]
        nb = n * self.max_blocks
        hd_np["block_tables"][:nb] = self.np["block_tables"][:nb]
        end = self._dec_bt_off + nb * 4
        if self._h2d_kernel:
            # a kernel reading the pinned buffer's device mapping: the step's next kernel
            # follows it on the stream without the idle gap a hipMemcpyAsync H2D left
            torch.ops.akap.h2d_stage(self.ddec[:end], self.hdecs[slot][:end])
        else:
            self.ddec[:end].copy_(self.hdecs[slot][:end], non_blocking=True)
        return slot

    def _h2d(self, key: str, n: int) -> torch.Tensor:
        dst = self.d[key][:n]
        dst.copy_(self.h[key][:n], non_blocking=True)
        return dst

    # ------------------------------------------------------------------ execution
    def _sample(self, logits: torch.Tensor, n: int, extras: Optional[dict] = None,
                src: Optional[dict] = None):
        """extras (from the engine, only when some request in the step asks for them):
        "penalties": (rows, toks, counts, presence, frequency, repetition) numpy COO over
        the sampled rows; "logprobs": True -> log-probs also for greedy picks."""
        lp = False
        if extras:
            pen = extras.get("penalties")
            if pen is not None:
                dev = logits.device
                rows, toks, counts, pres, freq, rep = pen
                ops.apply_penalties(
                    logits, torch.from_numpy(rows).to(dev), torch.from_numpy(toks).to(dev),
                    torch.from_numpy(counts).to(dev), torch.from_numpy(pres).to(dev),
                    torch.from_numpy(freq).to(dev), torch.from_numpy(rep).to(dev))
            lp = bool(extras.get("logprobs"))
        d = self.d if src is None else src
        ntop = int(extras.get("top_logprobs") or 0) if extras else 0
        if ntop > 0:
            # OpenAI top_logprobs: the N most likely tokens under the distribution the
            # sampler draws from (post-penalty logits, temperature-scaled when T > 0; the
            # same convention as the sampled token's log-prob)
            t = d["temperature"][:n].float()
            x = logits.float() / torch.where(t > 0, t, torch.ones_like(t))[:, None]
            vals, idx = torch.topk(x, min(ntop, x.shape[-1]), dim=-1)
            vals = vals - torch.logsumexp(x, dim=-1, keepdim=True)
            self.last_top = (idx.cpu().numpy(), vals.cpu().numpy())
        mode = self._sample_mode(n)
        return ops.sample(logits, d["temperature"][:n], d["top_k"][:n],
                          d["top_p"][:n], d["seeds"][:n], d["steps"][:n],
                          out_tokens=self.out_tokens[:n], out_logprobs=self.out_logprobs[:n],
                          greedy_logprobs=lp, filtered=mode == "filtered",
                          greedy_only=mode == "greedy" and not lp)

    def _sample_mode(self, n: int) -> str:
        """Sampler variant for the step's n sampled rows, from the host staging arrays:
        "greedy" (every row at temperature 0: the argmax kernel), "filtered" (some row uses
        top-k / top-p: the threshold passes), else "plain".  Inside a capture, the variant
        being captured; multi-rank engines always run "filtered" (correct for every batch)."""
        if self._capture_mode is not None:
            return self._capture_mode
        if not self.is_gpu or self._peer_step:
            return "filtered"
        npd, V = self.np, self.mcfg.vocab_size
        t, k, p = npd["temperature"][:n], npd["top_k"][:n], npd["top_p"][:n]
        if not (t > 0).any():
            return "greedy"
        if ((t > 0) & (((k > 0) & (k < V)) | ((p > 0) & (p < 1)))).any():
            return "filtered"
        return "plain"

    def _graph_for(self, n: int, B: int):
        """The decode graph of bucket n for a batch of B rows in its sampler mode (all modes
        were captured with the buckets; see capture_graphs)."""
        g = self.graphs.get(n)
        if g is None or self._peer_step:
            return g
        mode = self._sample_mode(B)
        return g if mode == "plain" else self.graphs_v[(mode, n)]

    PREFILL_FIELDS = ("input_ids", "positions", "slots", "seq_lens", "q_start", "block_tables",
                      "tile_seq", "tile_row", "logits_idx", "temperature", "top_p", "top_k",
                      "seeds", "steps", "tail_slot")

    def _prefill_extents(self, info: dict) -> dict:
        T, B, nt, ns = info["num_tokens"], info["num_seqs"], info["num_tiles"], info["num_samples"]
        return {"input_ids": T, "positions": T, "slots": T, "seq_lens": B, "q_start": B + 1,
                "block_tables": B * self.max_blocks, "tile_seq": nt, "tile_row": nt,
                "logits_idx": ns, "temperature": ns, "top_p": ns, "top_k": ns, "seeds": ns,
                "steps": ns, "tail_slot": T}

    def _stage_prefill(self, info: dict) -> dict:
        """The used prefix of every step buffer packed into ONE pinned region -> ONE H2D copy
        (instead of 14 small copies, each a blit kernel + host launch); under TP that one
        device region is then RCCL-broadcast from the group's rank 0 (over xGMI), so the
        other ranks never receive prefill payloads over the host control channel.  Returns
        device views per field."""
        ext = self._prefill_extents(info)
        lay, off = {}, 0
        for k in self.PREFILL_FIELDS:
            nb = ext[k] * self.h[k].element_size()
            lay[k] = (off, ext[k])
            off += -(-nb // 16) * 16
        end = off
        if self._hpre is None or self._hpre.numel() < end:
            cap = max(end, 1 << 16)
            self._hpre = self._pinned(cap, torch.uint8)
            self._dpre = torch.zeros(cap, dtype=torch.uint8, device=self.device)
        tp = self._tp_bcast_inputs
        if not (tp and self.ps.tp_rank != 0):
            hb = self._hpre.numpy()
            for k in self.PREFILL_FIELDS:
                o, n = lay[k]
                if n:
                    src = self.np[k][:n].view(np.uint8)
                    hb[o:o + src.size] = src
            self._dpre[:end].copy_(self._hpre[:end], non_blocking=True)
        if tp:
            import torch.distributed as dist

            dist.broadcast(self._dpre[:end], src=self.ps.rank - self.ps.tp_rank,
                           group=self.ps.tp_group)
        return {k: self._dpre[o:o + n * self.h[k].element_size()].view(self.h[k].dtype)
                for k, (o, n) in lay.items()}

    def execute_prefill(self, info: dict) -> torch.Tensor:
        """A step with prefill chunks; under mixed batching its leading `num_decode` rows are
        running sequences' decode tokens (eager, same forward)."""
        T, B, nt, ns = info["num_tokens"], info["num_seqs"], info["num_tiles"], info["num_samples"]
        mb = self.max_blocks
        v = self._stage_prefill(info)
        ids, pos, slots = v["input_ids"], v["positions"], v["slots"]
        sl, qs, ts, tr, lidx = v["seq_lens"], v["q_start"], v["tile_seq"], v["tile_row"], \
            v["logits_idx"]
        bt = v["block_tables"].view(B, mb)
        nd = info.get("num_decode", 0)
        parts, ps = self.decode_partitions(nd) if nd else (1, 512)
        batch = AttnBatch(True, pos, slots, bt, sl, qs, ts, tr, parts, ps,
                          self.workspace, tile_rows=info.get("tile_rows") or self.tile_rows,
                          num_decode=nd,
                          v_tails=self.v_tails, tail_slot=v["tail_slot"])
        if self._ep_moe:
            moe_mod.ep_overflow_reset(self.device)
        h = self.model.forward(ids, batch, self.k_caches, self.v_caches)
        if self._ep_moe:
            # the fixed-capacity EP dispatch costs this step ONE host check, not a sync per MoE
            # layer: on an overflow (any rank) every rank re-runs the forward on the exact path
            # (same KV slots rewritten, same inputs)
            moe_mod.ep_overflow_reduce(self.device)
            if self._ep_overflowed():
                self.ep_overflow_steps += 1
                with moe_mod.exact_dispatch():
                    h = self.model.forward(ids, batch, self.k_caches, self.v_caches)
        if self.ps.world_size > 1:
            from ..parallel import comm

            comm.check_deferred()
        if ns == 0:
            # a chunk that samples nothing (a long prompt's inner chunk): the caller's
            # device->host copy of zero tokens does not wait for the GPU, but the H2D copies
            # above read the pinned host buffers when they EXECUTE -- finish them before the
            # scheduler rewrites those buffers for the next step (else the next step's ids /
            # slots leak into this chunk's KV)
            if self.is_gpu:
                torch.cuda.current_stream().synchronize()
            return self.out_tokens[:0]
        logits = self.model.compute_logits(h.index_select(0, lidx))
        if not self.is_gpu:
            logits = logits.float()  # the GPU sampler reads bf16 logits directly
        toks, _ = self._sample(logits, ns, info.get("extras"), src=v)
        return toks

    def decode_partitions(self, n: int) -> tuple[int, int]:
        """Split-KV plan for a decode batch of n sequences.  Enough (seq, kv-head)
        workgroups to fill 256 CUs (>= 8 per CU) -> no split (no reduce kernel, no partial
        traffic; measured 5.4 vs 5.0 TB/s at B=256); otherwise split the context so the
        grid reaches ~2048 workgroups."""
        wgs = n * self.model.hkv
        max_len = self.ecfg.max_model_len
        if wgs >= 2048:
            parts = 1
        else:
            parts = min(math.ceil(2048 / wgs), max(1, math.ceil(max_len / 256)))
        # a partition is at most ops.DECODE_MAX_PART tokens (the kernel holds one block id
        # per 128-token wave step in a VGPR lane: 64 steps)
        parts = max(parts, math.ceil(max_len / ops.DECODE_MAX_PART))
        ps = math.ceil(math.ceil(max_len / parts) / 128) * 128
        parts = math.ceil(max_len / ps)
        return parts, ps

    @property
    def _tp_bcast_inputs(self) -> bool:
        """TP: rank 0's staged decode inputs reach the other ranks by one RCCL broadcast of
        the staging region at the start of the decode step (captured in the graph), so a
        decode step costs the host control channel only the small step header."""
        return self.ps.tp_size > 1 and self.ps.tp_group is not None

    def _decode_body(self, n: int, extras: Optional[dict] = None) -> None:
        if self._tp_bcast_inputs:
            from ..parallel import comm

            comm.tp_broadcast(self.ddec)  # custom IPC broadcast (or RCCL), in the graph
        dd = self.dd
        if self._ep_moe:
            moe_mod.ep_overflow_reset(self.device)
        parts, ps = self.decode_partitions(n)
        batch = AttnBatch(False, dd["positions"][:n], dd["slots"][:n], self.dd_bt[:n],
                          dd["seq_lens"][:n], self.d["q_start"][:n + 1], None, None,
                          parts, ps, self.workspace, v_tails=self.v_tails,
                          tail_slot=dd["tail_slot"][:n])
        h = self.model.forward(dd["input_ids"][:n], batch, self.k_caches, self.v_caches)
        # sampler reads bf16 logits directly (no [n, V] fp32 cast pass)
        logits = self.model.compute_logits(h)
        self._sample(logits, n, extras, src=dd)
        if self._ep_moe:
            moe_mod.ep_overflow_reduce(self.device)

    @property
    def _peer_step(self) -> bool:
        """Every step issues collectives with peer ranks (TP, or expert-parallel MoE over the
        job): all ranks must replay the same graph variant.  DP replicas and P/D roles share a
        torch.distributed world but run their steps alone (world_size > 1, tp_size == 1)."""
        return self.ps.tp_size > 1 or self._ep_moe

    def _err_probe(self, slot: int):
        """Enqueue an async copy of the custom IPC collectives' error word to pinned host
        memory behind this step's kernels (None when the step runs no IPC collective).  A
        replayed graph cannot raise: a peer that never arrived only sets that word, and the
        step's sums are then stale -- the host checks it before the tokens are used."""
        car = self.ps.car
        if car is None or not self.is_gpu or not self._peer_step:
            return None
        h = self._err_host[slot]
        h.copy_(car.err_word, non_blocking=True)
        return h

    @staticmethod
    def _check_err(h) -> None:
        if h is not None and int(h[0]) != 0:
            from ..parallel.comm import CollectiveTimeout

            raise CollectiveTimeout(
                "custom IPC collective timed out in a decode step (a peer rank stalled): the "
                "step's tokens are discarded and the engine is marked unhealthy")

    def _check_follower_err(self) -> None:
        """TP followers do not wait for their steps: check the newest probe whose copy has
        completed (a lag of a step or two), so a follower that summed stale staging stops
        before its corrupted KV writes feed later steps."""
        pend = self._follower_err
        while pend and pend[0][0].query():
            ev, h = pend.pop(0)
            self._check_err(h)

    @property
    def _ep_moe(self) -> bool:
        """Expert-parallel MoE layers over more than one rank (fixed-capacity dispatch)."""
        return self.ps.world_size > 1 and any(
            getattr(getattr(layer, "moe", None), "mode", None) == "ep"
            for layer in getattr(self.model, "layers", []))

    def _ep_overflowed(self) -> bool:
        """After a replayed decode step: did a fixed-capacity EP dispatch drop a pair on any
        rank?  (all-reduced inside the step, so every rank answers the same)"""
        return self._ep_moe and int(moe_mod.MoEBlock.overflow_flag(self.device).item()) != 0

    def _pad_host(self, B: int, n: int) -> None:
        if n <= B:
            return
        npd = self.np
        npd["input_ids"][B:n] = 0
        npd["positions"][B:n] = 0
        npd["slots"][B:n] = -1
        npd["seq_lens"][B:n] = 0
        npd["temperature"][B:n] = 0.0
        npd["top_p"][B:n] = 1.0
        npd["top_k"][B:n] = 0
        npd["seeds"][B:n] = 0
        npd["steps"][B:n] = 0
        npd["src_rows"][B:n] = 0
        npd["tail_slot"][B:n] = -1

    def execute_decode(self, info: dict) -> torch.Tensor:
        B = info["num_seqs"]
        n = B
        graph = None
        if self.graphs:
            for b in self.buckets:
                if b >= B:
                    n, graph = b, self.graphs[b]
                    break
        if not (self._tp_bcast_inputs and self.ps.tp_rank != 0):
            self._pad_host(B, n)
            self._stage_decode(n)  # (other TP ranks receive it by the in-graph broadcast)
        extras = info.get("extras")
        if graph is not None and not extras:
            if not (self._tp_bcast_inputs and self.ps.tp_rank != 0):
                graph = self._graph_for(n, B)
            graph.replay()
        else:
            # penalties / log-probs requested: the same padded batch (n rows, so TP peers
            # replaying their graphs issue identical collectives), eagerly
            self._decode_body(n, extras)
        self._ep_rerun_if_overflowed(n, extras)
        if self.ps.world_size > 1:
            from ..parallel import comm

            comm.check_deferred()
        self._pending_err = self._err_probe(2)
        return self.out_tokens[:B]

    def _ep_rerun_if_overflowed(self, n: int, extras: Optional[dict]) -> None:
        """After a decode step (replayed or eager): routing skew beyond the fixed dispatch
        capacity on any rank -> every rank redoes the step eagerly on the exact-split path (the
        same KV slots are rewritten, the tokens replaced)."""
        if self._ep_overflowed():
            self.ep_overflow_steps += 1
            with moe_mod.exact_dispatch():
                self._decode_body(n, extras)

    def launch_decode(self, info: dict, chained: bool = False):
        """Queue a graph-replayed decode step without waiting for it.  chained: the step was
        built by Scheduler.schedule_lookahead while the previous decode step is still
        queued -- its input ids are gathered on the device from that step's sampled tokens
        (out_tokens[src_rows]) before the replay (under TP only rank 0 gathers: the replay's
        first op broadcasts rank 0's staging region, gathered ids included, to the group).
        Returns a handle for wait_decode().  Without graphs (CPU) the step runs eagerly and
        the handle holds its tokens (same protocol, no overlap)."""
        B = info["num_seqs"]
        n, graph = B, None
        for b in self.buckets:
            if b >= B:
                n, graph = b, self.graphs[b]
                break
        if graph is None and self.is_gpu:
            raise RuntimeError(f"no decode graph holds {B} rows")
        self._pad_host(B, n)
        with profiling.phase("akap.decode"):
            slot = self._stage_decode(n)
            if chained:
                torch.index_select(self.out_tokens[:self.max_seqs], 0, self.dd["src_rows"][:n],
                                   out=self.dd["input_ids"][:n])
            if graph is not None:
                self._graph_for(n, B).replay()
            else:
                self._decode_body(n)
        if not self.is_gpu:
            return None, self.out_tokens[:B].clone(), self._err_probe(slot)
        host = self.tok_host[slot][:B]
        host.copy_(self.out_tokens[:B], non_blocking=True)
        err = self._err_probe(slot)
        ev = torch.cuda.Event()
        ev.record()
        return ev, host, err

    def replay_decode(self, info: dict) -> None:
        """TP follower ranks: the decode step's graph replay alone -- inputs arrive by the
        in-graph broadcast of rank 0's staging region, nobody on this rank needs the tokens,
        so nothing is staged and the host does not wait (the next header finds the GPU
        still busy with this step, not idle behind a host round trip)."""
        B = info["num_seqs"]
        n, graph = B, None
        for b in self.buckets:
            if b >= B:
                n, graph = b, self.graphs[b]
                break
        self._replays += 1
        if graph is not None:
            if self._replays != _FAULT_SKIP_REPLAY:  # fault injection (tests): skip one step
                graph.replay()
        else:
            self._decode_body(n)
        if self.is_gpu and self.ps.car is not None:
            self._check_follower_err()
            slot = self._follower_slot = (self._follower_slot + 1) % 4
            h = self._err_probe(3 + slot)
            if h is not None:
                ev = torch.cuda.Event()
                ev.record()
                self._follower_err.append((ev, h))

    def _bucket(self, B: int) -> int:
        for b in self.buckets:
            if b >= B:
                return b
        return B

    def execute_decode_eager(self, info: dict) -> None:
        """TP follower ranks, for a decode step rank 0 runs eagerly (its extras: penalties /
        log-probs): the same padded batch through _decode_body, so this rank issues exactly
        the collectives rank 0 does (inputs by the in-step broadcast of rank 0's staging
        region; an expert-parallel overflow re-run happens on every rank alike)."""
        n = self._bucket(info["num_seqs"])
        self._decode_body(n)
        self._ep_rerun_if_overflowed(n, None)

    @classmethod
    def wait_decode(cls, handle) -> np.ndarray:
        ev, host, err = handle
        if ev is not None:
            ev.synchronize()
        cls._check_err(err)  # never hand out tokens of a step whose collectives timed out
        return host.numpy()

    def execute(self, info: dict) -> np.ndarray:
        if info["is_prefill"]:
            with profiling.phase("akap.prefill"):
                toks = self.execute_prefill(info)
        else:
            with profiling.phase("akap.decode"):
                toks = self.execute_decode(info)
        if info["is_prefill"]:
            self._pending_err = self._err_probe(2)
        extras = info.get("extras")
        if extras and extras.get("logprobs"):
            self.last_logprobs = self.out_logprobs[:toks.shape[0]].to("cpu").numpy()
        out = toks.to("cpu").numpy()  # blocking: the probe copy queued before it is done
        err, self._pending_err = self._pending_err, None
        self._check_err(err)
        return out

    # ------------------------------------------------------------------ graphs
    def _graph_has_collectives(self) -> bool:
        """TP ranks and expert-parallel MoE layers issue RCCL calls inside the decode graph
        (DP replicas and single-GPU engines do not)."""
        if self.ps.world_size > 1:
            return True
        return any(getattr(getattr(layer, "moe", None), "mode", None) == "ep"
                   for layer in getattr(self.model, "layers", []))

    def capture_graphs(self) -> None:
        maxbs = min(self.ecfg.cuda_graph_max_bs or self.max_seqs, self.max_seqs)
        self.buckets = [b for b in DEFAULT_BUCKETS if b <= maxbs]
        if not self.buckets or self.buckets[-1] < maxbs:
            self.buckets.append(maxbs)
        t0 = time.time()
        tunable = os.environ.get("AKAP_TUNABLEOP", "0") == "1"
        if tunable:
            # PyTorch-ROCm TunableOp: benchmark hipBLASLt/rocBLAS solutions for every decode
            # GEMM shape once, before capture (the graph then bakes in the winner).
            torch.cuda.tunable.enable(True)
            torch.cuda.tunable.tuning_enable(True)
            torch.cuda.tunable.set_max_tuning_iterations(30)
            torch.cuda.tunable.set_filename(os.environ.get(
                "AKAP_TUNABLEOP_FILE", os.path.join(os.getcwd(), "tunableop_results.csv")))
        # safe static contents: every row is padding
        self._pad_host(0, self.max_seqs)
        if os.environ.get("AKAP_GEMM_TUNE", "1") != "0":
            # MoE models: the attention projections are tuned (the experts run the grouped
            # GEMM; tune_fused skips MoE layers)
            # per-(M, N, K) hipBLASLt vs MFMA-kernel choice on the real, cold layer weights
            from ..ops import gemm_tuner

            t1 = time.time()
            tune_ms = [b for b in self.buckets if b >= 16]
            cache = os.environ.get("AKAP_GEMM_TUNE_CACHE")
            if cache and self.model.ps.world_size > 1:
                cache = f"{cache}.rank{self.model.ps.rank}"
            pre_m = self.ecfg.max_num_batched_tokens
            loaded = bool(cache) and gemm_tuner.load_cache(cache, self.model, tune_ms, pre_m)
            if self.ps.tp_size > 1:
                # tune_fused broadcasts rank 0's plan over the TP group: every rank must take
                # the same branch, so one rank's missing / stale cache file retunes them all
                from ..parallel import comm

                agreed = comm.tp_all_true(loaded)
                if loaded and not agreed:
                    gemm_tuner.reset()
                loaded = agreed
            if loaded:
                self.log(f"[runner] GEMM plan loaded from {cache} "
                         f"({len(gemm_tuner.plan())} shapes)")
            else:
                gemm_tuner.tune_model(self.model, tune_ms, log=self.log)
                if os.environ.get("AKAP_FUSED_GEMM", "1") != "0":
                    gemm_tuner.tune_fused(self.model, tune_ms, log=self.log)
                if ops.PREFILL_GEMM == "auto" and pre_m >= ops.PGEMM_MIN_M:
                    gemm_tuner.tune_prefill(self.model, pre_m, log=self.log)
                if cache:
                    gemm_tuner.save_cache(cache, self.model, tune_ms, pre_m)
            self.log(f"[runner] GEMM tuning {time.time() - t1:.1f}s")
        self._stage_decode(self.max_seqs)
        torch.cuda.synchronize()
        if self._peer_step:
            # the warm-up steps below run the custom IPC collectives, whose flag waits are
            # bounded (~2 s): a rank still tuning its prefill GEMMs (rank-local, tens of seconds
            # at 70B widths) would time them out on its peers -- meet first.  Only the ranks
            # that share the step's collectives meet (the TP group; the whole job for
            # expert-parallel MoE): DP replicas and P/D roles capture on their own
            import torch.distributed as dist

            dist.barrier(group=None if self._ep_moe else self.ps.tp_group)
        self.graph_pool = torch.cuda.graph_pool_handle()
        stream = torch.cuda.Stream()
        # one graph per bucket and sampler mode (single-rank engines: "plain", "greedy" and
        # "filtered", all captured here -- a capture while serving would race the P/D KV
        # receiver's work; multi-rank engines: "filtered" only, correct for every batch)
        modes = ["filtered"] if self._peer_step else ["plain", "greedy", "filtered"]
        for mode in modes:
            self._capture_mode = mode
            for b in reversed(self.buckets):
                with torch.cuda.stream(stream):
                    self._decode_body(b)  # warm-up (hipBLASLt heuristics, allocator)
                stream.synchronize()
                if self._graph_has_collectives():
                    drain_pending_collectives(self.ps)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self.graph_pool, stream=stream):
                    self._decode_body(b)
                if mode == modes[0]:
                    self.graphs[b] = g
                else:
                    self.graphs_v[(mode, b)] = g
        self._capture_mode = None
        torch.cuda.synchronize()
        if tunable:
            torch.cuda.tunable.tuning_enable(False)
        self.log(f"[runner] captured {len(self.graphs)} decode hipGraphs "
                 f"(bs {self.buckets[0]}..{self.buckets[-1]}) in {time.time() - t0:.1f}s")
