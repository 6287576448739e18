"""Per-shape decode-GEMM dispatch: hipBLASLt vs the hand-written MFMA GEMM (csrc/kernels/
gemm.hip) at its best split-K, chosen by measurement at engine start.

Decode GEMMs read every layer's weights once per step, cold (the KV stream has evicted
them), and at M = batch they are latency/issue bound rather than bandwidth bound, so the
winner depends on (M, N, K): measured on MI355X, Llama-3-8B's down projection at M=128 is
49 us with the MFMA kernel at split-K 8 vs 75 us in hipBLASLt, while hipBLASLt wins the
wide gate|up projection (`profiles/r1_gemm_splitk_sweep.log`).  PyTorch TunableOp cannot
make this choice: it only ranks hipBLASLt/rocBLAS solutions, and it times them on warm
weights.

The tuner times each candidate on the model's REAL per-layer weights, rotating through
all layers inside one captured hipGraph (so every call sees cold weights, as in a decode
step), and records the winner in the plan `ops.linear` consults.  Candidates: hipBLASLt, the
MFMA GEMM at each split-K, and the k-pipelined decode GEMM (csrc/kernels/dgemm.hip, plain
prologue) at each (split-K, prefetch depth) -- the latter wins the narrow-N projections
(o-proj, N = d) where a block's K loop is a chain of round trips
(`profiles/r1_dgemm_micro.log`).
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

Choice = tuple  # ("torch",) | ("hip", splitk) | ("dgemm", splitk, prefetch_depth[, lds_dma_bn,
#                 ring_slots, in_launch_combine]) | ("wgemm",)
_PLAN: dict = {}

# positional defaults of a "dgemm" choice's variant fields after (split-K, prefetch):
# (LDS-DMA tile width, ring depth, in-launch combine, kgemm rows, tile rows)
VARIANT_DEFAULTS = (0, 0, False, 0, 64)


def variant_fields(v) -> tuple:
    """(bn, ns, inlaunch, km, bm) of a choice's tail, missing trailing fields defaulted."""
    v = tuple(v)
    return v + VARIANT_DEFAULTS[len(v):]


def plan() -> dict:
    return _PLAN


def reset() -> None:
    """Forget every tuned choice (per-shape plan, fused chains, prefill GEMM choices)."""
    _PLAN.clear()
    _FUSED.clear()
    _PREFILL.clear()


def lookup(M: int, N: int, K: int) -> Optional[Choice]:
    return _PLAN.get((M, N, K))


def _timed(fn, n: int) -> float:
    """us per call of fn(i), i < n, measured on a captured graph replay."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(min(n, 2)):
            fn(i)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    # best of three 2-replay windows: a candidate's time is its undisturbed time, so one
    # noisy window cannot hand the plan to a slower variant
    best = float("inf")
    for _ in range(3):
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        g.replay()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best * 1000.0 / (2 * n)


def _timed_eager(fn, n: int) -> float:
    """us per call of fn(i), i < n, launched eagerly (for library calls that refuse stream
    capture, e.g. torch._grouped_mm)."""
    fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for i in range(n):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / n


def _gd_variants(s: int, bns, M: int = 0):
    """gdgemm.hip variants at split s: (tile width, ring depth, in-launch split-K combine, tile
    rows).  Depth 0 = shallow ring (two blocks per CU), 8 = deep ring (one block per CU);
    128 x 128 tiles (rows 128) have their own 4-slot ring; 256-row tiles (8 waves, 3-slot
    ring) once the batch needs more than one 128-row tile (M > 128: at M = 160 Llama-3-8B's
    gate_up takes 89 us on two 128-row tiles, 71 us for a whole 256-row batch on one).  (The 256-row 6-slot ring of
    32-deep k-steps, ns = 6, lost on every M = 256 shape: profiles/r3_gemm_m256_deep.log.)"""
    for bn in bns:
        for ns in (0, 8):
            for inl in ((False, True) if s > 1 else (False,)):
                yield bn, ns, inl, 64
        if bn == 128:
            for inl in ((False, True) if s > 1 else (False,)):
                yield bn, 4, inl, 128
        if M > 128:
            for inl in ((False, True) if s > 1 else (False,)):
                yield bn, 3, inl, 256


def _gd_call(M, N, K, s, bn, ns, inl, out, x, weights, epi, ss_in, ss_out, a_out, ln_out,
             bm=64):
    """fn(i) launching one gdgemm variant on weights[i % len] (workspace/tickets bound)."""
    from . import gdgemm_ws_floats, gemm_counters

    dev = x.device
    ws = torch.empty(max(1, gdgemm_ws_floats(M, N, s, bn, bm) if s > 1 else 1), device=dev,
                     dtype=torch.float32)
    cnt = gemm_counters(dev) if (inl and s > 1) else None
    n = len(weights)
    return lambda i: torch.ops.akap.dgemm(out, x, weights[i % n], ws, 0, s, 1, None, None, None,
                                          1e-6, epi, ss_in, ss_out, a_out, ln_out, bn, ns, cnt,
                                          bm)


def _rr_inl_ok(s: int) -> bool:
    """Time the register-ring in-launch combine at split s (AKAP_DGEMM_RR_INL=0: never, the
    round-5 candidate set, for A/Bs)."""
    import os

    return s in (2, 4, 8) and os.environ.get("AKAP_DGEMM_RR_INL", "1") != "0"


def _rr_inl_call(M, N, s, pf, out, x, weights, epi, ss_in, ss_out, a_out, ln_out):
    """fn(i): the register-ring dgemm with its s K slices combined inside the launch."""
    from . import gdgemm_ws_floats, gemm_counters

    ws = torch.empty(gdgemm_ws_floats(M, N, s, 64, 64), device=x.device, dtype=torch.float32)
    cnt = gemm_counters(x.device)
    n = len(weights)
    return lambda i: torch.ops.akap.dgemm(out, x, weights[i % n], ws, 0, s, pf, None, None, None,
                                          1e-6, epi, ss_in, ss_out, a_out, ln_out, 0, 0, cnt, 64)


def _rot(weights: Sequence[torch.Tensor], cold_bytes: int = 768 << 20) -> list:
    """The layer copies a candidate is timed on: enough to stream >= cold_bytes per rotation
    (3x the 256 MB MALL, so every call still sees cold weights) and at least 4, not all of
    them -- tuning time scales with the rotation (Llama-3-8B: 32 layers of 50-235 MB each)."""
    w = list(weights)
    if not w:
        return w
    per = w[0].numel() * w[0].element_size()
    return w[:max(4, min(len(w), -(-cold_bytes // max(1, per))))]


# choice rankings of the anchor batch sizes (shape class pruning, see tune_model)
_RANK: dict = {}


def _plain_candidates(M, weights, x, y, splits, pfs, bns, kms, lm_head):
    """(choice, fn) for every hand-written way to compute x[M, K] @ w.T (hipBLASLt apart)."""
    from . import dgemm_supported, kgemm_supported

    w0 = weights[0]
    N, K = w0.shape
    dev = w0.device
    n = len(weights)
    if K % 64 == 0:  # wide-row weight-streaming kernel (csrc/kernels/wgemm.hip)
        yield ("wgemm",), (lambda i: torch.ops.akap.wgemm(y, x, weights[i % n]))
    for s in (() if lm_head else splits):
        if K // s < 256 or K % (64 * s):
            continue
        ws = torch.empty(max(1, s * M * N), device=dev, dtype=torch.float32)
        yield ("hip", s), (lambda i, ws=ws, s=s: torch.ops.akap.gemm(y, x, weights[i % n], ws, s))
    for s in splits:
        for pf in pfs:
            if not dgemm_supported(M, N, K, s, pf) or (s > 1 and K // s < 256):
                continue
            ws = torch.empty(max(1, s * M * N), device=dev, dtype=torch.float32)
            yield ("dgemm", s, pf), (lambda i, ws=ws, s=s, pf=pf: torch.ops.akap.dgemm(
                y, x, weights[i % n], ws, 0, s, pf))
            if _rr_inl_ok(s):  # the same with the slices combined inside the launch
                yield (("dgemm", s, pf, 0, 0, True),
                       _rr_inl_call(M, N, s, pf, y, x, weights, 0, None, None, None, None))
        for bn, ns, inl, bm in _gd_variants(s, bns, M):  # LDS-DMA staged variants (gdgemm.hip)
            if (not dgemm_supported(M, N, K, s, 1, bn=bn, inlaunch=inl, bm=bm)
                    or (s > 1 and K // s < 256) or (lm_head and bm != 256)):
                continue
            yield (("dgemm", s, 1, bn, ns, inl, 0, bm),
                   _gd_call(M, N, K, s, bn, ns, inl, y, x, weights, 0, None, None, None, None,
                            bm))
    for km in kms:  # K split inside the workgroup (csrc/kernels/kgemm.hip)
        if not kgemm_supported(M, N, K, km):
            continue
        yield (("dgemm", 1, 1, 0, 0, False, km),
               lambda i, km=km: torch.ops.akap.kgemm(y, x, weights[i % n], km, 0, 1e-6, None,
                                                     None, None, None))


def tune(M: int, weights: Sequence[torch.Tensor], splits=(1, 2, 4, 8, 16),
         margin: float = 0.03, pfs=(2, 4, 8), bns=(64, 128), kms=(16, 32),
         lm_head: bool = False, allowed: Optional[set] = None) -> Choice:
    """Pick the fastest way to compute x[M, K] @ w.T for these same-shape weights.
    hipBLASLt is kept unless the MFMA kernel is more than `margin` faster.  lm_head: only the
    256-row LDS-DMA tiles among the gdgemm variants (the narrow ones re-stream the
    activations once per 64-128 of ~150k columns).  allowed: time only these choices (the
    shape-class pruning of tune_model); the ranking lands in _RANK[(M, N, K)]."""
    from . import gemm_counters  # noqa: F401  (ensures the native library is loaded)

    weights = _rot(weights)
    w0 = weights[0]
    N, K = w0.shape
    dev = w0.device
    x = torch.randn(M, K, device=dev, dtype=w0.dtype) * 0.1
    y = torch.empty(M, N, device=dev, dtype=w0.dtype)
    n = len(weights)
    t_torch = _timed(lambda i: torch.nn.functional.linear(x, weights[i % n]), n)
    timed = [(t_torch, ("torch",))]
    for choice, fn in _plain_candidates(M, weights, x, y, splits, pfs, bns, kms, lm_head):
        if allowed is not None and choice not in allowed:
            continue
        timed.append((_timed(fn, n), choice))
    timed.sort(key=lambda tc: tc[0])
    _RANK[(M, N, K)] = [c for _, c in timed]
    t_best, best = timed[0]
    if best[0] != "torch" and t_best > t_torch * (1.0 - margin):
        best = ("torch",)
    _PLAN[(M, N, K)] = best
    return best


def anchor_ms(Ms: Sequence[int]) -> list:
    """Batch sizes tuned over every candidate (AKAP_GEMM_TUNE_FULL=1: all of them): the
    smallest, 64, 128 and the largest bucket.  The others time only the top
    AKAP_GEMM_TUNE_TOP (3) choices of their two neighbouring anchors: the decode GEMMs fall
    into shape classes whose winning variant changes only at a few batch sizes (round-5
    plans: kgemm below 128 rows, register ring / 128-wide LDS-DMA tiles above), so the
    per-bucket search is mostly re-confirming a neighbour's pick (Llama-3-8B cold start
    128.8 s, profiles/r5 pd_llama8b)."""
    import os

    ms = sorted(set(int(m) for m in Ms))
    if os.environ.get("AKAP_GEMM_TUNE_FULL", "0") == "1" or len(ms) <= 4:
        return ms
    want = {ms[0], ms[-1]} | {m for m in (64, 128) if m in ms}
    return sorted(want)


def _neighbour_allowed(M: int, anchors: list, rank_of) -> Optional[set]:
    """Union of the top choices of the anchors just below and above M (None: M is an
    anchor)."""
    import os

    if M in anchors:
        return None
    top = int(os.environ.get("AKAP_GEMM_TUNE_TOP", "3"))
    lo = [a for a in anchors if a < M]
    hi = [a for a in anchors if a > M]
    allowed: set = set()
    for a in ([lo[-1]] if lo else []) + ([hi[0]] if hi else []):
        allowed.update(rank_of(a)[:top])
    return allowed


def _gd_name(v) -> str:
    bn, ns, inl, km, bm = variant_fields(v)[:5]
    if km:
        return f"k{km}"
    if not bn:  # register ring (prefetch depth printed by the caller)
        return "i" if inl else ""
    if bm in (128, 256):
        return f"g{bn}x{bm}" + ("i" if inl else "")
    return f"g{bn}" + ("d" if ns >= 6 else "") + ("i" if inl else "")


def tune_model(model, Ms: Sequence[int], log=print) -> dict:
    """Tune every dense projection shape of `model` (per layer type) for each M."""
    groups = {}
    for lw in model.layers:
        for name in ("w_qkv", "w_o", "w_gate_up", "w_down"):
            w = getattr(lw, name, None)
            if w is not None:
                groups.setdefault((name, tuple(w.shape)), []).append(w)
    summary = {}
    anchors = anchor_ms(Ms)
    order = anchors + [m for m in sorted(set(Ms)) if m not in anchors]
    for M in order:
        for (name, shape), ws in groups.items():
            N, K = shape
            allowed = _neighbour_allowed(M, anchors,
                                         lambda a, N=N, K=K: _RANK.get((a, N, K), []))
            summary[(M, name)] = tune(M, ws, allowed=allowed)
    lm = getattr(model, "lm_head", None)
    if lm is not None and lm.is_cuda:
        # the decode LM head: hipBLASLt vs the wide-row kernel (split-K slabs of a vocab-wide
        # output would be GBs); at M > 160 also the 256-row LDS-DMA tiles without split-K
        # (every weight byte crosses L2 -> CU once)
        for M in Ms:
            big = M > 160
            summary[(M, "lm_head")] = tune(M, [lm], splits=(1,) if big else (), pfs=(),
                                           bns=(128,) if big else (), kms=(), lm_head=True)
    wins = {k: v for k, v in summary.items() if v[0] != "torch"}
    log(f"[gemm-tuner] {len(summary)} decode GEMM shapes, HIP kernel chosen for "
        f"{len(wins)}: " + ", ".join(
            f"M={m} {n} {c[0]}" + (f" s{c[1]}" if len(c) > 1 else "") +
            (f"p{c[2]}" if len(c) == 3 or (len(c) > 3 and not c[3] and
                                          not variant_fields(c[3:])[3]) else "") +
            (_gd_name(c[3:]) if len(c) > 3 else "")
            for (m, n), c in sorted(wins.items())))
    return summary


# ----------------------------------------------------------------------------- fused decode chain
# A dense decode layer as 4 fused GEMM launches (csrc/kernels/dgemm.hip epilogues):
#   qkv      plain, rows scaled by the input norm's rsqrt       (ss_in)
#   o        residual += y; a2 = residual * ln2; ss2 += row sum  (EPI_RESNORM)
#   gate_up  plain with ss2 row scale, SwiGLU epilogue           (EPI_SILU)
#   down     residual += y; a1' = residual * ln1'; ss1' += ...   (EPI_RESNORM)
# vs the unfused 7 launches (2 fused_add_rms_norm + silu_and_mul + 4 GEMMs at their tuned
# best).  Chosen per M when the fused chain measures faster.
_FUSED: dict = {}
_FUSED_ROLES = (("w_qkv", 0), ("w_o", 1), ("w_gate_up", 2), ("w_down", 1))  # (weight, epi)


def fused_plan(M: int) -> Optional[dict]:
    return _FUSED.get(M)


def _time_unfused(M: int, model) -> float:
    lw0 = model.layers[0]
    d = lw0.w_o.shape[0]
    F = lw0.w_down.shape[1]
    dev = lw0.w_o.device
    x = torch.randn(M, d, device=dev, dtype=lw0.w_o.dtype) * 0.1
    res = torch.randn(M, d, device=dev, dtype=lw0.w_o.dtype)
    h = torch.empty_like(x)
    gu = torch.randn(M, 2 * F, device=dev, dtype=lw0.w_o.dtype)
    act = torch.empty(M, F, device=dev, dtype=lw0.w_o.dtype)
    n = 8
    t_norm = _timed(lambda i: torch.ops.akap.fused_add_rmsnorm(h, res, x, lw0.ln1, 1e-6), n)
    t_silu = _timed(lambda i: torch.ops.akap.silu_and_mul(act, gu), n)
    return 2 * t_norm + t_silu


def tune_fused(model, Ms: Sequence[int], log=print, splits=(1, 2, 4, 8), pfs=(2, 4, 8),
               verbose: Optional[bool] = None, bns=(64, 128), kms=(16, 32)) -> dict:
    """Pick (split-K, prefetch) for each fused-chain GEMM at each M and keep the fused chain
    for the M where it beats the unfused chain (both timed on the real cold layer weights)."""
    from . import EPI_SILU, dgemm_supported, kgemm_supported

    if not model.layers or any(getattr(l, "moe", None) is not None for l in model.layers):
        return {}
    if verbose is None:  # AKAP_GEMM_TUNE_VERBOSE=1: per-role winners and runners-up
        import os

        verbose = os.environ.get("AKAP_GEMM_TUNE_VERBOSE", "0") == "1"
    L = len(model.layers)
    dev = model.layers[0].w_o.device
    dt = model.layers[0].w_o.dtype
    chosen = {}
    # tensor parallel: O / down store partial sums (their residual epilogue runs in the
    # all-reduce, comm.tp_all_reduce_resnorm), so they are timed with the plain store
    roles = _FUSED_ROLES if model.ps.tp_size == 1 else tuple(
        (n, 0 if n in ("w_o", "w_down") else e) for n, e in _FUSED_ROLES)
    anchors = anchor_ms(Ms)
    franks: dict = {}  # (M, name) -> candidate tuples by time (anchors only)
    order = anchors + [m for m in sorted(set(Ms)) if m not in anchors]
    for M in order:
        t_unfused = _time_unfused(M, model)
        plan_m, t_fused = {}, 0.0
        detail = []
        for name, epi in roles:
            allowed = _neighbour_allowed(M, anchors,
                                         lambda a, name=name: franks.get((a, name), []))
            timed_c: list = []
            ws_ = _rot([getattr(l, name) for l in model.layers])
            L = len(ws_)
            N, K = ws_[0].shape
            t_plain = _time_best_plain(M, name, ws_)
            t_unfused += t_plain
            x = torch.randn(M, K, device=dev, dtype=dt) * 0.1
            out = (torch.randn(M, N, device=dev, dtype=dt) if epi == 1 else
                   torch.empty(M, N // 2 if epi == EPI_SILU else N, device=dev, dtype=dt))
            ss = torch.full((M,), float(K), device=dev, dtype=torch.float32)
            ss_o = torch.zeros(M, device=dev, dtype=torch.float32)
            a_o = torch.empty(M, N, device=dev, dtype=dt)
            ln = model.layers[0].ln2 if N == model.layers[0].ln2.numel() else None
            best = None
            ss_in_, ss_out_ = (None if epi == 1 else ss), (ss_o if epi == 1 else None)
            a_o_, ln_ = (a_o if epi == 1 else None), (ln if epi == 1 else None)
            for s in splits:
                cands = [(pf, 0, 0, False, 0, 64) for pf in pfs] + \
                    [(pf, 0, 0, True, 0, 64) for pf in pfs if _rr_inl_ok(s)] + \
                    [(1, bn, ns, inl, 0, bm) for bn, ns, inl, bm in _gd_variants(s, bns, M)]
                if s == 1:
                    cands += [(1, 0, 0, False, km, 64) for km in kms
                              if kgemm_supported(M, N, K, km, epi)]
                for pf, bn, ns, inl, km, bm in cands:
                    if allowed is not None and (s, pf, bn, ns, inl, km, bm) not in allowed:
                        continue
                    if km:
                        fn = (lambda i, km=km: torch.ops.akap.kgemm(
                            out, x, ws_[i % L], km, epi, 1e-6, ss_in_, ss_out_, a_o_, ln_))
                        t = _timed(fn, L)
                        timed_c.append((t, (s, pf, bn, ns, inl, km, bm)))
                        if best is None or t < best[0]:
                            best = (t, s, pf, bn, ns, inl, km, bm)
                        continue
                    if (not dgemm_supported(M, N, K, s, pf, epi, bn=bn, inlaunch=inl, bm=bm)
                            or (s > 1 and K // s < 256)):
                        continue
                    if bn:
                        fn = _gd_call(M, N, K, s, bn, ns, inl, out, x, ws_, epi, ss_in_,
                                      ss_out_, a_o_, ln_, bm)
                    elif inl:
                        fn = _rr_inl_call(M, N, s, pf, out, x, ws_, epi, ss_in_, ss_out_, a_o_,
                                          ln_)
                    else:
                        wsp = torch.empty(max(1, s * M * N), device=dev, dtype=torch.float32)
                        fn = (lambda i, s=s, pf=pf, wsp=wsp: torch.ops.akap.dgemm(
                            out, x, ws_[i % L], wsp, 0, s, pf, None, None, None, 1e-6, epi,
                            ss_in_, ss_out_, a_o_, ln_, 0))
                    t = _timed(fn, L)
                    timed_c.append((t, (s, pf, bn, ns, inl, 0, bm)))
                    if best is None or t < best[0]:
                        best = (t, s, pf, bn, ns, inl, 0, bm)
            franks[(M, name)] = [c for _, c in sorted(timed_c, key=lambda tc: tc[0])]
            if verbose:
                log(f"[gemm-tuner] M={M} {name} top: " + ", ".join(
                    f"{t:.2f}us s{c[0]}" + (_gd_name(c[2:]) if (c[2] or c[5]) else
                                          f"p{c[1]}" + ("i" if c[4] else ""))
                    for t, c in sorted(timed_c, key=lambda tc: tc[0])[:5]))
            if best is None:
                plan_m = None
                break
            plan_m[name] = best[1:]
            t_fused += best[0]
            detail.append(f"{name} {best[0]:.1f}/{t_plain:.1f} (s{best[1]}"
                          + (_gd_name(best[3:]) if (best[3] or best[6]) else
                             f"p{best[2]}" + ("i" if best[5] else ""))
                          + ")")
        if plan_m is not None and t_fused < t_unfused:
            _FUSED[M] = plan_m
        chosen[M] = (t_fused, t_unfused, plan_m)
        if verbose:
            log(f"[gemm-tuner] M={M} fused/plain us: " + ", ".join(detail))
    if model.ps.tp_size > 1:
        # every TP rank must run the same chain (the same collectives per step): rank 0's
        # timing decides
        from ..parallel import comm

        import torch.distributed as dist

        g = model.ps.tp_group
        plans = comm.broadcast_object({m: _FUSED.get(m) for m in Ms},
                                      src=dist.get_global_rank(g, 0) if g is not None else 0,
                                      group=g)
        for m, pl in plans.items():
            if pl is None:
                _FUSED.pop(m, None)
            else:
                _FUSED[m] = pl
    used = [m for m in Ms if m in _FUSED]
    log("[gemm-tuner] fused decode layer chain (us/layer fused vs unfused): " + ", ".join(
        f"M={m} {c[0]:.1f}/{c[1]:.1f}" + ("*" if m in _FUSED else "")
        for m, c in sorted(chosen.items())) + f"  -> fused for {len(used)} of {len(Ms)} "
        f"batch sizes (full search at M={anchors})")
    return chosen


# ----------------------------------------------------------------------------- prefill GEMMs
# Prefill-sized projections (M = the prefill chunk, thousands of rows): hipBLASLt vs the
# hand-written 256 x 256 pgemm (csrc/kernels/pgemm.hip), per weight shape, with the SwiGLU
# epilogue variant for gate|up (pgemm + fused epilogue vs hipBLASLt + silu_and_mul) and the
# expert-grouped form for MoE layers (pgemm over device offsets vs torch._grouped_mm).
# Keys: ("dense", N, K, silu) | ("grouped", N, K, silu) -> True when pgemm measured faster.
_PREFILL: dict = {}


def prefill_choice(kind: str, N: int, K: int, silu: bool = False) -> Optional[bool]:
    return _PREFILL.get((kind, N, K, bool(silu)))


def tune_prefill(model, M: int, log=print, margin: float = 0.02) -> dict:
    """Time both paths for every prefill projection shape of `model` at M rows, on the real
    layer weights (rotating through the layers inside one captured graph)."""
    from . import pgemm_supported, silu_and_mul

    groups: dict = {}
    for lw in model.layers:
        for name in ("w_qkv", "w_o", "w_gate_up", "w_down"):
            w = getattr(lw, name, None)
            if w is not None and w.is_cuda:
                groups.setdefault(tuple(w.shape) + (name == "w_gate_up",), []).append(w)
    out = {}
    dev = None
    for (N, K, gu), ws in groups.items():
        if not pgemm_supported(M, N, K):
            continue
        dev = ws[0].device
        x = torch.randn(M, K, device=dev, dtype=ws[0].dtype) * 0.1
        y = torch.empty(M, N, device=dev, dtype=ws[0].dtype)
        n = len(ws)
        t_lib = _timed(lambda i: torch.matmul(x, ws[i % n].t(), out=y), n)
        t_pg = _timed(lambda i: torch.ops.akap.pgemm(y, x, ws[i % n], 0, None), n)
        _PREFILL[("dense", N, K, False)] = t_pg < t_lib * (1.0 - margin)
        out[("dense", N, K, False)] = (t_pg, t_lib)
        if gu:
            a = torch.empty(M, N // 2, device=dev, dtype=ws[0].dtype)
            t_lib_s = _timed(lambda i: silu_and_mul(torch.matmul(x, ws[i % n].t(), out=y), a), n)
            t_pg_s = _timed(lambda i: torch.ops.akap.pgemm(a, x, ws[i % n], 2, None), n)
            _PREFILL[("dense", N, K, True)] = t_pg_s < t_lib_s * (1.0 - margin)
            out[("dense", N, K, True)] = (t_pg_s, t_lib_s)
        del x, y
    for lw in model.layers:  # MoE experts: one representative layer
        moe = getattr(lw, "moe", None)
        if moe is None or not moe.w13.is_cuda:
            continue
        E = moe.w13.shape[0]
        rows = M * moe.K
        g = torch.Generator(device="cpu").manual_seed(0)
        cnt = torch.multinomial(torch.ones(E), rows, replacement=True,
                                generator=g).bincount(minlength=E)
        offs = cnt.cumsum(0).to(torch.int32).to(moe.w13.device)
        for w, silu in ((moe.w13, True), (moe.w2, False)):
            _, N, K = w.shape
            if not pgemm_supported(rows, N, K):
                continue
            x = torch.randn(rows, K, device=w.device, dtype=w.dtype) * 0.1
            o = torch.empty(rows, N // 2 if silu else N, device=w.device, dtype=w.dtype)
            wt = w.transpose(1, 2)
            if silu:
                lib = lambda i: silu_and_mul(torch._grouped_mm(x, wt, offs=offs), o)  # noqa: E731
            else:
                lib = lambda i: torch._grouped_mm(x, wt, offs=offs)  # noqa: E731
            t_lib = _timed_eager(lib, 3)
            t_pg = _timed_eager(lambda i: torch.ops.akap.pgemm(o, x, w, 2 if silu else 0, offs),
                                3)
            _PREFILL[("grouped", N, K, silu)] = t_pg < t_lib * (1.0 - margin)
            out[("grouped", N, K, silu)] = (t_pg, t_lib)
            del x, o
        break
    if out:
        log(f"[gemm-tuner] prefill GEMMs at M={M} (us pgemm/library): " + ", ".join(
            f"{k[0]} {k[1]}x{k[2]}{' silu' if k[3] else ''} {a:.0f}/{b:.0f}"
            + ("*" if _PREFILL[k] else "") for k, (a, b) in out.items()))
    return out


# ----------------------------------------------------------------------------- tuning cache
# The plan is a pure function of (GPU, kernel library, model shapes, TP layout, batch
# buckets): a JSON file keyed on those lets a restarted engine skip the ~3-10 s of timing
# (AKAP_GEMM_TUNE_CACHE=path, engine/model_runner.py), and keeps a profiled run free of the
# tuning candidates' launches.  Any key mismatch -> retune and overwrite.
CACHE_VERSION = 2


def cache_key(model, Ms: Sequence[int], prefill_m: int = 0) -> dict:
    import os

    from . import _LIB

    shapes = sorted({(name, tuple(getattr(lw, name).shape)) for lw in model.layers
                     for name in ("w_qkv", "w_o", "w_gate_up", "w_down")
                     if getattr(lw, name, None) is not None})
    lm = getattr(model, "lm_head", None)
    try:
        arch = torch.cuda.get_device_properties(0).gcnArchName if torch.cuda.is_available() \
            else "cpu"
    except Exception:  # pragma: no cover - device query failures
        arch = "unknown"
    try:
        st = os.stat(_LIB)
        lib = [st.st_size, int(st.st_mtime)]
    except OSError:
        lib = None
    return {"version": CACHE_VERSION, "arch": arch, "lib": lib,
            "tp": [model.ps.tp_size, model.ps.tp_rank], "layers": len(model.layers),
            "shapes": [[n, list(sh)] for n, sh in shapes],
            "lm_head": list(lm.shape) if lm is not None else None, "Ms": sorted(int(m) for m in Ms),
            "prefill_m": int(prefill_m)}


def save_cache(path: str, model, Ms: Sequence[int], prefill_m: int = 0) -> None:
    import json
    import os

    data = {"key": cache_key(model, Ms, prefill_m),
            "plan": [[list(k), list(v)] for k, v in sorted(_PLAN.items())],
            "fused": [[m, {n: list(t) for n, t in pl.items()}] for m, pl in sorted(_FUSED.items())],
            "prefill": [[list(k), v] for k, v in sorted(_PREFILL.items())]}
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "w") as f:
        json.dump(data, f)
    os.replace(tmp, path)  # readers never see a half-written file


def load_cache(path: str, model, Ms: Sequence[int], prefill_m: int = 0) -> bool:
    """Install the cached plan when its key matches this model/GPU/library; False otherwise."""
    import json

    try:
        with open(path) as f:
            data = json.load(f)
    except (OSError, ValueError):
        return False
    if data.get("key") != cache_key(model, Ms, prefill_m):
        return False
    plan_ = {tuple(k): tuple(v) for k, v in data["plan"]}
    fused_ = {int(m): {n: tuple(t) for n, t in pl.items()} for m, pl in data["fused"]}
    # the 256 x 256 stream-K body (bn = 256, pgemm_sk) is probe-only: a combine that times
    # out there only sets GEMM_CTR_ERR, which no serving step reads -- never serve it from a
    # (hand-edited or foreign) cache file
    if any(c[0] == "dgemm" and len(c) > 3 and variant_fields(c[3:])[0] == 256
           for c in plan_.values()) or any(
            len(e) > 2 and variant_fields(e[2:])[0] == 256
            for pl in fused_.values() for e in pl.values()):
        return False
    _PLAN.clear()
    _FUSED.clear()
    _PLAN.update(plan_)
    _FUSED.update(fused_)
    _PREFILL.clear()
    for k, v in data.get("prefill", []):
        _PREFILL[tuple(k)] = bool(v)
    return True


def _time_best_plain(M: int, name: str, weights) -> float:
    """us of the plan's choice for this projection (hipBLASLt unless tuned otherwise)."""
    weights = _rot(weights)
    w0 = weights[0]
    N, K = w0.shape
    x = torch.randn(M, K, device=w0.device, dtype=w0.dtype) * 0.1
    c = _PLAN.get((M, N, K), ("torch",))
    n = len(weights)
    if c[0] == "dgemm":
        y = torch.empty(M, N, device=w0.device, dtype=w0.dtype)
        if len(c) > 6 and c[6]:
            return _timed(lambda i: torch.ops.akap.kgemm(y, x, weights[i % n], c[6], 0, 1e-6, None,
                                                         None, None, None), n)
        if len(c) > 3 and c[3]:
            bn, ns, inl, _, bm = variant_fields(c[3:])[:5]
            return _timed(_gd_call(M, N, K, c[1], bn, ns, inl, y, x, weights, 0, None, None,
                                   None, None, bm), n)
        if len(c) > 5 and c[5]:
            return _timed(_rr_inl_call(M, N, c[1], c[2], y, x, weights, 0, None, None, None,
                                       None), n)
        ws = torch.empty(max(1, c[1] * M * N), device=w0.device, dtype=torch.float32)
        return _timed(lambda i: torch.ops.akap.dgemm(y, x, weights[i % n], ws, 0, c[1], c[2],
                                                     None, None, None, 1e-6, 0, None, None,
                                                     None, None, 0), n)
    if c[0] == "wgemm":
        y = torch.empty(M, N, device=w0.device, dtype=w0.dtype)
        return _timed(lambda i: torch.ops.akap.wgemm(y, x, weights[i % n]), n)
    if c[0] == "hip":
        ws = torch.empty(max(1, c[1] * M * N), device=w0.device, dtype=torch.float32)
        y = torch.empty(M, N, device=w0.device, dtype=w0.dtype)
        return _timed(lambda i: torch.ops.akap.gemm(y, x, weights[i % n], ws, c[1]), n)
    return _timed(lambda i: torch.nn.functional.linear(x, weights[i % n]), n)
