"""Mixture-of-experts FFN (Mixtral, Qwen3-MoE) with tensor-parallel or expert-parallel experts.

Routing is the HIP `moe_topk_softmax` kernel; token grouping is `moe_align` (expert-
sorted, tile-padded index list).  Two placements:
  * "tp": every rank holds all experts with the FFN dim split by tp (one all-reduce,
    like a dense layer) -- best at small batch on a single xGMI node;
  * "ep": rank e holds experts [e*E/ep, (e+1)*E/ep) whole; tokens are dispatched and
    combined with two all-to-alls over the EP (=dp x tp) group (the custom IPC kernel at
    decode sizes when the TP group spans the job, else RCCL all_to_all_single).
Expert GEMMs: `ops.fused_moe` -- device-side sort + grouped MFMA GEMMs + gather-combine,
no host sync, at every batch size in "tp" mode (decode steps inside the hipGraph, prefill
chunks eagerly); the per-expert loop below serves only the CPU reference path.

"ep" mode: a FIXED-CAPACITY dispatch -- every (token, expert) pair gets a slot (destination
rank, rank-local index) computed on the device, the send buffer is [ep, C, d] with
C = ep_capacity(n) = max(ceil(slack * n / ep), min(n, 8)) for the n = T*K pairs of this rank
(slack 2 by default, AKAP_EP_SLACK): the exchanged bytes stay within slack x the exact n*d
however many ranks there are, where a worst-case C = n would move ep*n*d.  Both
all_to_all_single calls use equal splits and no split size goes to the host, so the whole EP
MoE block (route, dispatch, grouped expert GEMMs on the received rows, combine) is sync-free
and graph-capturable.  Empty slots carry expert id -1: moe_align skips them at decode sizes,
and at prefill sizes they sort into a dummy group past the last expert offset that the
grouped GEMM never computes.  A pair whose destination already holds C pairs (a routing skew
the capacity does not cover) is not sent; it raises the shared overflow flag instead, which
the STEP all-reduces over the EP group at its end (ep_overflow_reduce) and checks once on the
host: the runner then re-runs that step under exact_dispatch() (ModelRunner.execute_prefill /
execute_decode), so an overflow costs one extra step, never a wrong token, and a prefill
step no longer pays a host sync per MoE layer.  The exact path (split sizes to the host, one
sync per layer) serves those re-runs, and eager steps above AKAP_EP_FIXED_MAX_T tokens
(0 = always exact: tests).
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch
import torch.nn.functional as F

from .. import ops
from ..parallel import comm
from ..parallel.state import ParallelState


def ep_overflow_reset(device) -> None:
    MoEBlock.overflow_flag(device).zero_()


def ep_overflow_reduce(device) -> torch.Tensor:
    """All-reduce (MAX) of the fixed-dispatch overflow flag over the EP group: every rank
    sees the same value, so all of them re-run an overflowed step together."""
    f = MoEBlock.overflow_flag(device)
    if torch.distributed.is_initialized():
        from ..parallel.state import get_state

        st = get_state()
        if st is not None and st.car is not None and st.tp_size == st.world_size:
            # inside a captured decode step: the custom IPC all-reduce (a bf16 sum of 0/1 flags
            # is exact for <= 8 ranks), no process-group collective in the graph
            b = f.to(torch.bfloat16).repeat(8)
            st.car.all_reduce(b)
            f.copy_(torch.gt(b[:1], 0).to(torch.int32))
        else:
            torch.distributed.all_reduce(f, op=torch.distributed.ReduceOp.MAX)
    return f


@contextlib.contextmanager
def exact_dispatch():
    """Re-run a step whose fixed-capacity dispatch overflowed: every EP layer inside takes the
    exact-split path.  Counted in MoEBlock.ep_fallbacks."""
    MoEBlock.ep_fallbacks += 1
    MoEBlock.force_exact = True
    try:
        yield
    finally:
        MoEBlock.force_exact = False


class MoEBlock:
    def __init__(self, cfg, ps: ParallelState, device, dtype, g: torch.Generator,
                 full_then_shard: bool, mode: Optional[str] = None, std: float = 0.02):
        self.cfg = cfg
        self.ps = ps
        self.device = device
        self.dtype = dtype
        self.E = cfg.num_experts
        self.K = cfg.experts_per_token
        self.mode = mode or os.environ.get("AKAP_MOE_MODE", "tp")
        d, Fn = cfg.hidden_size, cfg.intermediate_size
        tp, r = ps.tp_size, ps.tp_rank

        def rand(*shape):
            t = torch.empty(*shape, dtype=torch.float32, device=g.device)
            t.normal_(0.0, std, generator=g)
            return t.to(dtype)

        if self.mode == "ep":
            ep = ps.world_size
            if self.E % ep:
                raise ValueError("num_experts must divide by the EP size")
            self.ep, self.ep_rank = ep, ps.rank
            self.e_local = self.E // ep
            self.e0 = self.ep_rank * self.e_local
            self.f_local = Fn
        else:
            self.ep, self.ep_rank = 1, 0
            self.e_local, self.e0 = self.E, 0
            self.f_local = Fn // tp
        self.router = rand(self.E, d).to(device)
        if full_then_shard:
            w1 = rand(self.E, Fn, d)
            w3 = rand(self.E, Fn, d)
            w2 = rand(self.E, d, Fn)
            if self.mode == "ep":
                sl = slice(self.e0, self.e0 + self.e_local)
                w13 = torch.cat([w1[sl], w3[sl]], 1)
                w2s = w2[sl]
            else:
                fs = slice(r * self.f_local, (r + 1) * self.f_local)
                w13 = torch.cat([w1[:, fs], w3[:, fs]], 1)
                w2s = w2[:, :, fs]
            self.w13 = w13.contiguous().to(device)
            self.w2 = w2s.contiguous().to(device)
        else:
            self.w13 = rand(self.e_local, 2 * self.f_local, d).to(device)
            self.w2 = rand(self.e_local, d, self.f_local).to(device)

    def numel(self) -> int:
        return self.router.numel() + self.w13.numel() + self.w2.numel()

    def _hf_names(self, prefix: str, e: int) -> tuple:
        """HF checkpoint names: (router, gate, up, down) of expert e -- Mixtral's
        block_sparse_moe.{gate, experts.e.w1/w3/w2} or Qwen3-MoE's mlp.{gate,
        experts.e.gate_proj/up_proj/down_proj}."""
        if self.cfg.arch == "qwen3_moe":
            p = f"{prefix}mlp.experts.{e}."
            return (prefix + "mlp.gate.weight", p + "gate_proj.weight", p + "up_proj.weight",
                    p + "down_proj.weight")
        p = f"{prefix}block_sparse_moe.experts.{e}."
        return (prefix + "block_sparse_moe.gate.weight", p + "w1.weight", p + "w3.weight",
                p + "w2.weight")

    def load_state_dict(self, sd: dict, prefix: str) -> None:
        r, tp = self.ps.tp_rank, self.ps.tp_size
        self.router.copy_(sd[self._hf_names(prefix, 0)[0]])
        for j in range(self.e_local):
            e = self.e0 + j
            _, n1, n3, n2 = self._hf_names(prefix, e)
            w1, w3, w2 = sd[n1], sd[n3], sd[n2]
            if self.mode != "ep":
                fs = slice(r * self.f_local, (r + 1) * self.f_local)
                w1, w3, w2 = w1[fs], w3[fs], w2[:, fs]
            self.w13[j].copy_(torch.cat([w1, w3], 0))
            self.w2[j].copy_(w2)

    def hf_state_dict(self, prefix: str) -> dict:
        """HF names (Mixtral or Qwen3-MoE) of this unsharded block's router and experts."""
        if self.e_local != self.E or self.f_local != self.cfg.intermediate_size:
            raise ValueError("hf_state_dict needs the unsharded MoE block")
        Fn = self.f_local
        sd = {self._hf_names(prefix, 0)[0]: self.router.clone()}
        for e in range(self.E):
            _, n1, n3, n2 = self._hf_names(prefix, e)
            sd[n1] = self.w13[e, :Fn].clone()
            sd[n3] = self.w13[e, Fn:].clone()
            sd[n2] = self.w2[e].clone()
        return sd

    def forward(self, h: torch.Tensor) -> torch.Tensor:
        if self.mode == "ep" and self.ps.tp_size > 1:
            # activations are replicated across the TP group: each rank routes only its
            # 1/tp token slice through the EP all-to-all, then the slices are all-gathered
            T = h.shape[0]
            tp, r = self.ps.tp_size, self.ps.tp_rank
            per = (T + tp - 1) // tp
            pad = per * tp - T
            hp = torch.cat([h, h.new_zeros(pad, h.shape[1])]) if pad else h
            mine = self._forward_tokens(hp[r * per:(r + 1) * per].contiguous())
            full = torch.empty(per * tp, h.shape[1], dtype=h.dtype, device=h.device)
            comm.tp_all_gather_rows(full, mine)
            return full[:T]
        return self._forward_tokens(h)

    ep_fixed_max_tokens = int(os.environ.get("AKAP_EP_FIXED_MAX_T", str(1 << 30)))
    ep_slack = float(os.environ.get("AKAP_EP_SLACK", "2.0"))
    # prefill-sized dispatches (>= 4096 pairs): the per-destination count concentrates near
    # the mean (sd ~ sqrt(n)), so a smaller slack halves the exchanged bytes at ep = 2; an
    # unusually skewed step overflows into the exact re-run
    ep_slack_prefill = float(os.environ.get("AKAP_EP_SLACK_PREFILL", "1.25"))
    ep_min_cap = int(os.environ.get("AKAP_EP_MIN_CAP", "8"))
    ep_fallbacks = 0  # steps re-run on the exact path after a dispatch overflow
    force_exact = False  # set by exact_dispatch() around such a re-run
    ep_exact_layers = 0  # layer calls on the exact (host-synced) path
    _overflow: dict = {}  # device -> int32 [1]: a fixed-capacity dispatch dropped a pair

    def ep_capacity(self, n: int) -> int:
        """Rows per destination rank in the fixed-capacity dispatch of n (token, expert) pairs:
        slack x the mean share, at least min(n, ep_min_cap = 8) (tiny decode batches), at most n."""
        import math

        slack = self.ep_slack if n < 4096 else min(self.ep_slack, self.ep_slack_prefill)
        return min(n, max(math.ceil(slack * n / self.ep), min(n, self.ep_min_cap)))

    @classmethod
    def overflow_flag(cls, device) -> torch.Tensor:
        key = str(device)
        if key not in cls._overflow:
            cls._overflow[key] = torch.zeros(1, dtype=torch.int32, device=device)
        return cls._overflow[key]

    @property
    def graph_safe(self) -> bool:
        """Decode steps capture in a hipGraph: tp mode (fused_moe) and ep mode (fixed-capacity
        dispatch) are both free of host syncs at decode sizes."""
        return True

    def _forward_tokens(self, h: torch.Tensor) -> torch.Tensor:
        T, d = h.shape
        w, ids = ops.moe_router_topk(h, self.router, self.K,
                                     renormalize=self.cfg.moe_renormalize)
        capturing = h.is_cuda and torch.cuda.is_current_stream_capturing()
        if self.mode == "ep":
            if capturing:
                return self._ep_fixed(h, w, ids)
            if T <= self.ep_fixed_max_tokens and not MoEBlock.force_exact:
                # no host sync here: an overflow only raises the shared flag, which the step
                # checks once at its end (ModelRunner) and answers with an exact re-run
                return self._ep_fixed(h, w, ids)
            return self._ep_exact(h, w, ids)
        # tp mode, no host sync at any size: decode sizes (and every captured step) on the
        # hand-written fused_moe, prefill sizes (and the CPU path) on the library grouped GEMM
        if h.is_cuda and (T < self.grouped_min_t or capturing):
            out = ops.fused_moe(h, self.w13, self.w2, w, ids)
        else:
            src = torch.arange(T * self.K, device=h.device) // self.K
            if h.is_cuda:
                # expert-sorted rows straight into the weighted combine (moe_combine gathers
                # each token's K rows through inv): no permutation store of the [T*K, d] rows
                ys, order = self._expert_rows(h, ids.reshape(-1), src, sorted_out=True)
                inv = torch.empty_like(order, dtype=torch.int32)
                inv[order] = torch.arange(order.numel(), dtype=torch.int32, device=h.device)
                out = torch.empty(T, d, dtype=h.dtype, device=h.device)
                torch.ops.akap.moe_combine(ys, w.float().contiguous(), inv, out)
            else:
                y = self._expert_rows(h, ids.reshape(-1), src)
                out = (y.view(T, self.K, d).float() * w.view(T, self.K, 1).float()).sum(1)
                out = out.to(h.dtype)
        comm.tp_all_reduce(out)
        return out

    grouped_min_t = int(os.environ.get("AKAP_MOE_GROUPED_MIN_T", "512"))

    def _expert_rows(self, x: torch.Tensor, e: torch.Tensor,
                     src: Optional[torch.Tensor] = None, sorted_out: bool = False):
        """y[i] = expert e[i]'s SwiGLU FFN of x[src[i]] (src = identity when None), unweighted.
        Rows are sorted by expert on the device (ids -1 = empty rows, skipped) and run through a grouped GEMM over device-side
        group offsets -- the hand-written pgemm (SwiGLU fused into the first GEMM's epilogue) or
        torch._grouped_mm (the ROCm library grouped GEMM), whichever measured faster at engine
        start (gemm_tuner.tune_prefill): no host sync, no per-expert loop.  Mixtral-8x7B shapes
        on MI355X: 1081 TFLOP/s at T=16384 and 847 at T=4096, vs
        617 / 444 for fused_moe and level with the host-synced per-expert hipBLASLt loop it
        replaces (profiles/r3_moe_prefill.log).  Outputs come back in row order (a permutation
        store: deterministic, no float atomics), or with sorted_out as (expert-sorted rows,
        order) for a caller that gathers them itself."""
        e = e.reshape(-1).long()
        el = self.e_local
        # empty fixed-dispatch slots (id -1) sort last into a dummy group past the final offset:
        # the grouped GEMM never computes those rows (their outputs are never read)
        key = torch.where(e < 0, torch.full_like(e, el), e)
        ks, order = torch.sort(key, stable=True)
        # group end offsets by binary search on the sorted ids: no bincount (its CUDA path reads
        # the max id back to the host)
        offs = torch.searchsorted(ks, torch.arange(el, device=ks.device, dtype=ks.dtype),
                                  right=True).to(torch.int32)
        xs = x[order if src is None else src[order]]
        if ops.use_pgemm(xs, self.w13.shape[1], silu=True, grouped=True):
            # hand-written grouped GEMM with SwiGLU in its epilogue (csrc/kernels/pgemm.hip)
            a = ops.pgemm(xs, self.w13, silu=True, offs=offs)
        else:
            a = ops.silu_and_mul(torch._grouped_mm(xs, self.w13.transpose(1, 2), offs=offs))
        if ops.use_pgemm(a, self.w2.shape[1], grouped=True):
            y = ops.pgemm(a, self.w2, offs=offs)
        else:
            y = torch._grouped_mm(a, self.w2.transpose(1, 2), offs=offs)
        if sorted_out:
            return y, order
        out = torch.empty_like(y)
        out[order] = y
        return out

    def a2a_rows(self, T: int) -> int:
        """Rows this rank sends per all_to_all of the fixed dispatch (= rows received)."""
        return self.ep * self.ep_capacity(T * self.K)

    def _ep_fixed(self, h: torch.Tensor, w: torch.Tensor, ids: torch.Tensor,
                  flag: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Sync-free, capturable EP dispatch/combine with per-peer capacity ep_capacity(T*K)."""
        T, d = h.shape
        K, ep, el = self.K, self.ep, self.e_local
        n = T * K
        C = self.ep_capacity(n)
        # rows per destination per exchange chunk (C unless the message must be split: the
        # single-GPU gloo rehearsal's IPC staging); C rounded up to whole chunks
        R = comm.ep_chunk_rows(C, d + 8, h)
        C = -(-C // R) * R
        nck = C // R
        flat = ids.reshape(-1).long()                       # [n] global expert ids
        dest = flat // el                                   # owning rank
        onehot = F.one_hot(dest, ep).to(torch.int32)        # [n, ep]
        # rank-local index of each pair: an inclusive scan along n of the [ep, n] transpose
        # (an inner-dim scan; PyTorch's outer-dim scan of [n, ep] ran ~5 ms per prefill layer)
        incl = torch.cumsum(onehot.t().contiguous(), dim=1, dtype=torch.int32)
        slot = incl.gather(0, dest.view(1, -1)).view(-1).long() - 1
        fits = slot < C
        # chunk-major rows [nck, ep, R]: chunk k of the exchange is one contiguous block whose
        # segment p goes to rank p (nck = 1: the plain [ep, C] layout all_to_all_single takes);
        # overflowing pairs go to a dump row past the send buffer (never sent)
        pos = torch.where(fits, (slot // R * ep + dest) * R + slot % R,
                          torch.full_like(slot, ep * C))
        flag = self.overflow_flag(h.device) if flag is None else flag
        torch.maximum(flag, (~fits).any().to(torch.int32).view(1), out=flag)
        tok = torch.arange(n, device=h.device) // K
        # one message per row: the token's hidden vector plus 8 trailing bf16 slots whose
        # first two carry the int32 local expert id (-1 = empty slot, whose vector is never
        # read), so the dispatch is ONE all-to-all (the EP group is the whole job: dp x tp)
        send = h.new_empty(ep * C + 1, d + 8)
        ids_col = send[:, d:d + 2].view(torch.int32)  # [ep*C + 1, 1] view into the rows
        ids_col.fill_(-1)
        send[:, :d].index_copy_(0, pos, h[tok])
        ids_col.index_copy_(0, pos, (flat - dest * el).to(torch.int32).view(-1, 1))
        send = send[:ep * C]
        recv = torch.empty_like(send)
        comm.ep_all_to_all_equal(recv, send, chunks=nck)
        recv_x = recv[:, :d].contiguous()
        recv_e = recv[:, d:d + 2].contiguous().view(torch.int32).reshape(-1, 1)
        # every received row is one (token, local expert) pair: K = 1, weight 1 (the router
        # weight is applied by the sender at combine); empty slots (id -1) are skipped
        if (h.is_cuda and not torch.cuda.is_current_stream_capturing()
                and ep * C >= self.grouped_min_t * K):
            y = self._expert_rows(recv_x, recv_e)  # prefill sizes: the grouped GEMM
        else:
            ones = torch.ones(ep * C, 1, dtype=torch.float32, device=h.device)
            y = ops.fused_moe(recv_x, self.w13, self.w2, ones, recv_e)
        back = h.new_empty(ep * C + 1, d)
        back[ep * C].zero_()  # the dump row overflowing pairs read (weighted, so finite)
        comm.ep_all_to_all_equal(back[:ep * C], y.contiguous(), chunks=nck)
        mine = back.index_select(0, pos).view(T, K, d).float()
        return (mine * w.view(T, K, 1)).sum(1).to(h.dtype)

    def _ep_exact(self, h: torch.Tensor, w: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
        """Prefill-size EP: exact split sizes (one host sync for the counts), received rows
        through the grouped expert GEMM (no per-expert host loop)."""
        MoEBlock.ep_exact_layers += 1
        T, d = h.shape
        flat = ids.reshape(-1).long()
        order = torch.argsort(flat, stable=True)
        tok_of = order // self.K
        grp = None  # the EP group is the whole job (dp x tp ranks)
        owner = flat[order] // self.e_local
        send_counts = torch.bincount(owner, minlength=self.ep)
        recv_counts = torch.empty_like(send_counts)
        torch.distributed.all_to_all_single(recv_counts, send_counts, group=grp)
        sc, rc = torch.stack([send_counts, recv_counts]).tolist()
        x_recv = comm.all_to_all(h[tok_of], rc, sc, group=grp)
        e_recv = comm.all_to_all(flat[order].to(torch.int32), rc, sc, group=grp) - self.e0
        if x_recv.is_cuda and x_recv.shape[0] < self.grouped_min_t * self.K:
            ones = torch.ones(x_recv.shape[0], 1, dtype=torch.float32, device=h.device)
            y_recv = ops.fused_moe(x_recv, self.w13, self.w2, ones, e_recv.view(-1, 1))
        else:
            y_recv = self._expert_rows(x_recv, e_recv)
        y_back = comm.all_to_all(y_recv, sc, rc, group=grp)
        wt = w.reshape(-1)[order].to(torch.float32)
        out = torch.zeros(T, d, dtype=torch.float32, device=h.device)
        out.index_add_(0, tok_of, y_back.float() * wt[:, None])
        return out.to(h.dtype)
