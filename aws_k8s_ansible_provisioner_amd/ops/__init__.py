"""Python entry points of the gfx950 kernels.

Every op dispatches on the device of its inputs:
  * GPU tensors  -> the hand-written HIP kernel in ``_C.so`` (``torch.ops.akap.*``).
    If the extension is missing on a GPU box this RAISES -- there is no silent
    eager fallback on the GPU path.
  * CPU tensors  -> a plain PyTorch reference of the same op (used by the CPU test
    suite, the CPU mock engine and as the numerics oracle of the GPU tests).

Layouts shared with the kernels (see csrc/kernels/rope_cache.hip):
  K cache [num_blocks, Hkv, BS, D], V cache [num_blocks, Hkv, BS/8, D, 8] (8-token groups).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import reference as ref

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB = os.path.join(_PKG, "_C.so")
_loaded = False
_load_error: Optional[str] = None


def load_native(required: bool = False) -> bool:
    """Load ``_C.so`` (torch.ops.akap).  Returns True when available."""
    global _loaded, _load_error
    if _loaded:
        return True
    if not os.path.exists(_LIB):
        _load_error = f"{_LIB} not built (run python -m aws_k8s_ansible_provisioner_amd.build_ext)"
    else:
        stale = native_provenance()
        if stale.get("mismatch") and os.environ.get("AKAP_ALLOW_STALE_NATIVE") != "1":
            _load_error = (f"{_LIB} was built from other sources (library tree "
                           f"{stale['library'][:16]}, sources here {stale['sources'][:16]}): "
                           f"rebuild with python -m aws_k8s_ansible_provisioner_amd.build_ext")
        else:
            try:
                torch.ops.load_library(_LIB)
                _loaded = True
            except Exception as e:  # pragma: no cover - depends on the box
                _load_error = repr(e)
    if required and not _loaded:
        raise RuntimeError("native HIP kernels unavailable: " + str(_load_error))
    return _loaded


def native_provenance() -> dict:
    """The source-tree digest compiled into _C.so vs the digest of the sources beside it
    (build_ext.kernel_tree_hash): proves which sources the loaded library was built from."""
    import ctypes

    from .. import build_ext

    lib = ctypes.CDLL(_LIB, mode=getattr(os, "RTLD_LAZY", 1) | ctypes.RTLD_GLOBAL)
    try:
        f = lib.akap_build_hash
    except AttributeError:
        return {"library": "none", "sources": "?", "mismatch": True}
    f.restype = ctypes.c_char_p
    have = f().decode()
    want = build_ext.kernel_tree_hash() if os.path.exists(build_ext.CSRC) else have
    return {"library": have, "sources": want, "mismatch": have != want}


def native_available() -> bool:
    return load_native(False)


def _native(t: torch.Tensor) -> bool:
    if t.is_cuda:
        load_native(required=True)
        return True
    return False


# ----------------------------------------------------------------------------- norms
def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None):
    if out is None:
        out = torch.empty_like(x)
    if _native(x):
        torch.ops.akap.rmsnorm(out, x, w, eps)
        return out
    out.copy_(ref.rms_norm(x, w, eps))
    return out


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                       out: Optional[torch.Tensor] = None):
    """residual += x (in place); returns (rmsnorm(residual), residual)."""
    if out is None:
        out = torch.empty_like(x)
    if _native(x):
        torch.ops.akap.fused_add_rmsnorm(out, residual, x, w, eps)
        return out, residual
    r = (x.float() + residual.float()).to(x.dtype)
    residual.copy_(r)
    out.copy_(ref.rms_norm(r, w, eps))
    return out, residual


# ----------------------------------------------------------------------------- rope/cache
def qk_norm_rope_cache(qkv, q_out, k_cache, v_cache, positions, slots, cos_sin, q_w, k_w,
                       num_q_heads: int, num_kv_heads: int, eps: float, apply_rope: bool = True,
                       decode: bool = False, v_tail=None, tail_slot=None, num_decode: int = 0,
                       q_rows: int = -1):
    """decode=True: one new token per sequence (V written per token instead of by the
    prefill role's 64-token span scan).  v_tail / tail_slot (GPU, bf16 cache, span role):
    tokens of a group still partial after this step also go to their sequence's V tail, and
    a decode row (t < num_decode) completing a group writes the whole group from the tail
    (csrc/kernels/rope_cache.hip); the CPU reference ignores the tail (its cache is always
    complete).  q_rows >= 0 (GPU): q is written only for tokens < q_rows -- the prefill
    attention applies the q norm + RoPE of the others itself (paged_attention_prefill qprep);
    the CPU reference always writes every q row."""
    if _native(qkv):
        torch.ops.akap.qk_norm_rope_cache(qkv, q_out, k_cache, v_cache, positions, slots, cos_sin,
                                          q_w, k_w, num_q_heads, num_kv_heads, eps, apply_rope,
                                          decode, v_tail, tail_slot if v_tail is not None else None,
                                          num_decode, q_rows)
        return q_out
    ref.qk_norm_rope_cache(qkv, q_out, k_cache, v_cache, positions, slots, cos_sin, q_w, k_w,
                           num_q_heads, num_kv_heads, eps, apply_rope)
    return q_out


def reshape_and_cache(k, v, k_cache, v_cache, slots):
    if _native(k):
        torch.ops.akap.reshape_and_cache(k, v, k_cache, v_cache, slots)
        return
    ref.reshape_and_cache(k, v, k_cache, v_cache, slots)


# ----------------------------------------------------------------------------- mlp
def silu_and_mul(x: torch.Tensor, out: Optional[torch.Tensor] = None):
    F = x.shape[-1] // 2
    if out is None:
        out = torch.empty(*x.shape[:-1], F, dtype=x.dtype, device=x.device)
    if _native(x):
        torch.ops.akap.silu_and_mul(out, x)
        return out
    out.copy_(ref.silu_and_mul(x))
    return out


# ----------------------------------------------------------------------------- attention
def paged_attention_prefill(out, q, k_cache, v_cache, block_tables, seq_lens, q_start, tile_seq,
                            tile_row, gqa_group: int, scale: float, tile_rows: int = 128,
                            qprep=None):
    """tile_rows = flattened q rows per tile of the host tile map: 128 selects the flash-style
    LDS-tiled kernel (32x32x16 MFMA, 4 waves), 256 its 8-wave form (bf16 KV cache).
    qprep = (qkv, positions, cos_sin, q_w, eps) (GPU): the kernel reads the raw q rows from
    the QKV projection and applies the q RMSNorm + RoPE itself (q is then only read by the
    CPU reference, whose q is always fully written).  The kernel rotates token i of a chunk
    by its key index seq_len - q_len + i -- the invariant its causal mask already assumes and
    what `positions` holds for prefill tokens."""
    if _native(q) and qprep is not None:
        qkv, positions, cos_sin, q_w, eps = qprep
        if DEBUG_CHECKS:
            check_qprep_positions(positions, seq_lens, q_start, cos_sin.shape[0])
        torch.ops.akap.paged_attention_prefill_qprep(out, qkv, k_cache, v_cache, block_tables,
                                                     seq_lens, q_start, tile_seq, tile_row,
                                                     positions, cos_sin, q_w, gqa_group, scale,
                                                     eps, tile_rows)
        return out
    if _native(q):
        torch.ops.akap.paged_attention_prefill(out, q, k_cache, v_cache, block_tables, seq_lens,
                                               q_start, tile_seq, tile_row, gqa_group, scale,
                                               tile_rows)
        return out
    out.copy_(ref.paged_attention(q, k_cache, v_cache, block_tables, seq_lens, q_start, scale))
    return out


# AKAP_DEBUG_CHECKS=1: host-side invariant checks that cost a device sync (off in serving)
DEBUG_CHECKS = os.environ.get("AKAP_DEBUG_CHECKS", "0") == "1"


def check_qprep_positions(positions, seq_lens, q_start, table_rows: int) -> None:
    """The q-prep prefill kernel rotates token i of a sequence's chunk by its KEY index
    seq_len - q_len + i (it never reads `positions`): raise if any prefill token's position
    differs from that index (e.g. a future M-RoPE or shifted-position model), or if the
    rotary table has fewer rows than the largest key index."""
    qs = q_start.to("cpu", torch.int64)
    sl = seq_lens.to("cpu", torch.int64)
    pos = positions.to("cpu", torch.int64)
    for b in range(sl.numel()):
        n = int(qs[b + 1] - qs[b])
        if n <= 0:
            continue
        want = torch.arange(int(sl[b]) - n, int(sl[b]), dtype=torch.int64)
        got = pos[int(qs[b]):int(qs[b + 1])]
        if not torch.equal(got, want):
            raise ValueError(f"prefill q-prep: sequence {b} positions {got[:4].tolist()}... "
                             f"are not its key indices {want[:4].tolist()}...")
        if int(sl[b]) > table_rows:
            raise ValueError(f"prefill q-prep: key index {int(sl[b]) - 1} past the rotary "
                             f"table's {table_rows} rows")


# longest decode split-KV partition the kernel takes (csrc/kernels/kernels.h kDecodeMaxPart)
DECODE_MAX_PART = 8192


def paged_attention_decode(out, q, k_cache, v_cache, block_tables, seq_lens, gqa_group: int,
                           scale: float, workspace=None, num_parts: int = 1,
                           part_size: int = 512, q_start=None, v_tail=None, tail_slot=None):
    """v_tail / tail_slot: a sequence's still-partial last V group is read from its tail."""
    if _native(q):
        if workspace is None:
            B = seq_lens.numel()
            Hkv = k_cache.shape[1]
            workspace = decode_workspace(B, Hkv, gqa_group, num_parts, q.device)
        pm, pl, po = workspace
        torch.ops.akap.paged_attention_decode(out, q, k_cache, v_cache, block_tables, seq_lens,
                                              q_start, pm, pl, po, num_parts, part_size,
                                              gqa_group, scale, v_tail,
                                              tail_slot if v_tail is not None else None)
        return out
    if q_start is None:
        q_start = torch.arange(seq_lens.numel() + 1, dtype=torch.int32)
    out.copy_(ref.paged_attention(q, k_cache, v_cache, block_tables, seq_lens, q_start, scale))
    return out


def paged_attention_decode_fused(out, qkv, k_cache, v_cache, block_tables, seq_lens, positions,
                                 slots, cos_sin, q_w, k_w, gqa_group: int, scale: float,
                                 eps: float, workspace=None, num_parts: int = 1,
                                 part_size: int = 512, v_tail=None, tail_slot=None):
    """Decode attention that consumes the raw QKV projection: per-head q/k RMSNorm + RoPE
    and the new token's K/V cache write happen inside the attention kernel.
    out [B, Hq, D]; qkv [B, (Hq + 2 Hkv) * D].  With v_tail (bf16 cache) the new token's V
    goes to its sequence's tail row and the cache gets whole 8-token groups only."""
    if _native(qkv):
        if workspace is None:
            workspace = decode_workspace(seq_lens.numel(), k_cache.shape[1], gqa_group,
                                         num_parts, qkv.device)
        pm, pl, po = workspace
        torch.ops.akap.paged_attention_decode_fused(out, qkv, k_cache, v_cache, block_tables,
                                                    seq_lens, positions, slots, cos_sin, q_w, k_w,
                                                    pm, pl, po, num_parts, part_size, gqa_group,
                                                    scale, eps, v_tail,
                                                    tail_slot if v_tail is not None else None)
        return out
    B, Hq = out.shape[0], out.shape[1]
    q = torch.empty_like(out)
    ref.qk_norm_rope_cache(qkv[:B], q, k_cache, v_cache, positions, slots, cos_sin, q_w, k_w, Hq,
                           k_cache.shape[1], eps, True)
    q_start = torch.arange(B + 1, dtype=torch.int32)
    out.copy_(ref.paged_attention(q, k_cache, v_cache, block_tables, seq_lens, q_start, scale))
    return out


def decode_workspace(max_seqs: int, num_kv_heads: int, gqa_group: int, num_parts: int,
                     device) -> tuple:
    n = max(1, max_seqs * num_kv_heads * max(num_parts, 1) * gqa_group)
    pm = torch.empty(n, dtype=torch.float32, device=device)
    pl = torch.empty(n, dtype=torch.float32, device=device)
    po = torch.empty(n * 128 if num_parts > 1 else 1, dtype=torch.float32, device=device)
    return pm, pl, po


# ----------------------------------------------------------------------------- GEMM
_GEMM_MODE = os.environ.get("AKAP_GEMM", "torch")  # torch (hipBLASLt) | auto | hip
GEMM_MAX_M = int(os.environ.get("AKAP_GEMM_MAX_M", "512"))
# prefill-sized GEMMs: "auto" = per weight shape, whichever of hipBLASLt and the hand-written
# 256 x 256 pgemm (csrc/kernels/pgemm.hip) measured faster at engine start
# (gemm_tuner.tune_prefill); "pgemm" / "lib" force one.  PGEMM_MIN_M: smallest M routed to it.
PREFILL_GEMM = os.environ.get("AKAP_PREFILL_GEMM", "auto")
PGEMM_MIN_M = int(os.environ.get("AKAP_PGEMM_MIN_M", "1024"))


def pgemm_supported(M: int, N: int, K: int) -> bool:
    """Mirror of pgemm_supported (csrc/kernels/pgemm.hip) and the 2 GiB operand limit of its
    buffer-descriptor DMA (ops.cpp)."""
    return (M > 0 and N > 0 and N % 256 == 0 and K >= 64 and K % 64 == 0
            and M * K * 2 < 2 ** 31 and N * K * 2 < 2 ** 31)


def use_pgemm(x: torch.Tensor, N: int, silu: bool = False, grouped: bool = False) -> bool:
    """Route x [M, K] times an [N, K] weight (or a grouped [G, N, K] one) to pgemm?"""
    if not (x.is_cuda and x.dim() == 2 and x.stride(-1) == 1 and x.shape[0] >= PGEMM_MIN_M
            and pgemm_supported(x.shape[0], N, x.shape[1])):
        return False
    if PREFILL_GEMM == "pgemm":
        return True
    if PREFILL_GEMM == "auto":
        from . import gemm_tuner

        return bool(gemm_tuner.prefill_choice("grouped" if grouped else "dense", N, x.shape[1],
                                              silu))
    return False


def _use_pgemm(x: torch.Tensor, w: torch.Tensor, silu: bool = False) -> bool:
    return w.dim() == 2 and use_pgemm(x, w.shape[0], silu)


def linear_silu(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """silu(x @ gate.T) * (x @ up.T) for the [gate; up] weight w [2F, K]: one pgemm launch
    with the SwiGLU epilogue for prefill-sized M (no [M, 2F] intermediate round trip through
    HBM), else linear + silu_and_mul."""
    if _use_pgemm(x, w, silu=True):
        load_native(required=True)
        return pgemm(x, w, silu=True)
    return silu_and_mul(linear(x, w))


def linear(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x @ w.T.  Decode-sized M on the GPU -> the hand-written MFMA GEMM (small tiles +
    split-K to fill 256 CUs); large M (prefill) -> hipBLASLt via torch, or the hand-written
    256 x 256 pgemm where it measured faster (AKAP_PREFILL_GEMM)."""
    M = x.shape[0]
    split = None
    if _use_pgemm(x, w):
        load_native(required=True)
        return pgemm(x, w, out=out)
    if x.is_cuda and x.dim() == 2:
        from . import gemm_tuner

        choice = gemm_tuner.lookup(M, w.shape[0], w.shape[1])
        if choice is not None and choice[0] == "wgemm" and x.stride(-1) == 1:
            return wgemm(x, w, out=out)
        if choice is not None:  # measured at engine start (cold weights, real layers)
            if choice[0] == "dgemm" and x.stride(-1) == 1:
                bn, ns, inl, km, bm = gemm_tuner.variant_fields(choice[3:])[:5]
                return dgemm(x, w, PRO_PLAIN, choice[1], choice[2], out=out, bn=bn, ns=ns,
                             inlaunch=inl, km=km, bm=bm)
            split = choice[1] if choice[0] == "hip" else 0
    if split is None:
        use_hip = (x.is_cuda and _GEMM_MODE != "torch" and x.dim() == 2 and x.stride(-1) == 1
                   and (M <= GEMM_MAX_M or _GEMM_MODE == "hip") and x.shape[1] % 8 == 0
                   and w.shape[0] % 4 == 0)
    else:
        use_hip = split > 0 and x.stride(-1) == 1
    if not use_hip:
        y = torch.nn.functional.linear(x, w)
        if out is not None:
            out.copy_(y)
            return out
        return y
    load_native(required=True)
    N, K = w.shape
    if out is None:
        out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    s = split or gemm_splitk(M, N, K)
    if s > 1:
        ws = torch.empty(s * M * N, dtype=torch.float32, device=x.device)
    else:
        ws = _EMPTY_F32.get(x.device)
        if ws is None:
            ws = _EMPTY_F32[x.device] = torch.empty(1, dtype=torch.float32, device=x.device)
    torch.ops.akap.gemm(out, x, w, ws, s)
    return out


def wgemm(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x @ w.T by the wide-row weight-streaming kernel (csrc/kernels/wgemm.hip): one
    workgroup owns all (<= 256) rows of a column tile, so each weight byte crosses HBM -> CU
    once -- the decode LM head.  CPU: plain matmul."""
    M, N = x.shape[0], w.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    if not _native(x):
        out.copy_(torch.nn.functional.linear(x.float(), w.float()).to(out.dtype))
        return out
    torch.ops.akap.wgemm(out, x, w)
    return out


PRO_PLAIN, PRO_ADDNORM, PRO_SILU = 0, 1, 2
EPI_STORE, EPI_RESNORM, EPI_SILU = 0, 1, 2


def silu_interleave_perm(F: int) -> torch.Tensor:
    """Row order in which EPI_SILU reads a [gate (F rows); up (F rows)] weight: 16-row groups
    alternate gate / up of the same 16 features (virtual column v -> this row)."""
    v = torch.arange(2 * F)
    return ((v >> 4) & 1) * F + (v >> 5) * 16 + (v & 15)


def dgemm(x: torch.Tensor, w: torch.Tensor, pro: int = PRO_PLAIN, splitk: int = 1, pf: int = 2,
          residual: Optional[torch.Tensor] = None, residual_out: Optional[torch.Tensor] = None,
          ln: Optional[torch.Tensor] = None, eps: float = 1e-6,
          out: Optional[torch.Tensor] = None, epi: int = EPI_STORE,
          ss_in: Optional[torch.Tensor] = None, ss_out: Optional[torch.Tensor] = None,
          a_out: Optional[torch.Tensor] = None, ln_out: Optional[torch.Tensor] = None,
          bn: int = 0, ns: int = 0, inlaunch: bool = False, km: int = 0,
          bm: int = 64) -> torch.Tensor:
    """Fused decode GEMM (csrc/kernels/dgemm.hip): y = A @ w.T where A is produced from x by
    the prologue inside the GEMM's operand staging --
      PRO_PLAIN    A = x; with ss_in, rows of y are scaled by rsqrt(ss_in / K + eps)
      PRO_ADDNORM  s = x + residual (written to residual_out), A = rmsnorm(s) * ln
      PRO_SILU     x = [gate | up] ([M, 2K]), A = silu(gate) * up
    and an epilogue --
      EPI_STORE    out = bf16(y)
      EPI_RESNORM  out is the residual stream [M, N] (in/out): out = bf16(bf16(y) + out);
                   a_out = bf16(out * ln_out); ss_out += per-row sum of out^2 (caller zeroes)
      EPI_SILU     w = [gate; up] rows, out [M, N/2] = silu(y_gate) * y_up
    replacing the separate fused_add_rms_norm / silu_and_mul launches of a decode layer.
    bn = 64 | 128 selects the LDS-DMA staged variant (csrc/kernels/gdgemm.hip, 64 x bn tiles,
    plain prologue only); 0 the register-ring kernel (prefetch depth pf).  For bn > 0:
    ns >= 6 selects the deep LDS ring (one block per CU, ~7 k-steps in flight), and with
    splitk > 1 inlaunch=True combines the K slices inside the launch (last-arriver ticket,
    no separate reduce kernel; also allows split-K with the SwiGLU epilogue) -- for bn = 0
    too (register-ring kernel, plain prologue, splitk 2 | 4 | 8).
    bm = 128 (with bn = 128): 128-row LDS-DMA tiles (weights cross L2 -> CU half as often at
    M = 256; the large-weight projections); bm = 256 (bn 64 | 128, 8 waves): the whole
    256-row batch per tile, every weight byte crosses L2 -> CU once.
    bn = 256 (bm = 256) selects the 256 x 256 pgemm body with the K range split over
    `splitk` workgroups per tile and the slices combined inside the launch by every slice
    (csrc/kernels/pgemm.hip pgemm_sk_kernel; all epilogues, grid <= the CU count).  That
    variant is PROBE-ONLY: when its all-slices spin times out (slices not co-resident) it only
    sets counters[GEMM_CTR_ERR] -- read by gemm_ctr_error() in tests and probes, never by a
    serving step -- so the tuner never emits it and gemm_tuner.load_cache refuses plans
    naming it.
    km = 16 | 32 selects csrc/kernels/kgemm.hip instead: km x 32 output tiles with the K split
    over the workgroup's waves (plain prologue, store / residual epilogues, no split-K)."""
    M = x.shape[0]
    N, K = w.shape
    if out is None:
        out = torch.empty(M, N // 2 if epi == EPI_SILU else N, dtype=x.dtype, device=x.device)
    if not _native(x):
        if pro == PRO_ADDNORM:
            s = (x.float() + residual.float()).to(x.dtype)
            residual_out.copy_(s)
            a = ref.rms_norm(s, ln, eps)
        elif pro == PRO_SILU:
            a = ref.silu_and_mul(x)
        else:
            a = x
        y = torch.nn.functional.linear(a.float(), w.float())
        if pro == PRO_PLAIN and ss_in is not None:
            y = y * torch.rsqrt(ss_in[:M].float() / K + eps)[:, None]
        if epi == EPI_RESNORM:
            r = (y.to(x.dtype).float() + out.float()).to(x.dtype)
            out.copy_(r)
            a_out.copy_((r.float() * ln_out.float()).to(x.dtype))
            ss_out[:M] += r.float().pow(2).sum(-1)
        elif epi == EPI_SILU:
            out.copy_(ref.silu_and_mul(y.to(x.dtype)))
        else:
            out.copy_(y.to(out.dtype))
        return out
    if km:
        torch.ops.akap.kgemm(out, x, w, km, epi, eps, ss_in, ss_out, a_out, ln_out)
        return out
    counters = None
    if splitk > 1:
        inl = inlaunch and (bn or (pro == PRO_PLAIN and splitk in (2, 4, 8)))
        n = (gdgemm_ws_floats(M, N, splitk, bn or 64, bm if bn else 64) if (bn or inl) else
             splitk * M * N + (splitk * M if pro == PRO_ADDNORM else 0))
        ws = torch.empty(n, dtype=torch.float32, device=x.device)
        if inl or bn == 256:  # bn 256: the combine is always in the launch
            counters = gemm_counters(x.device)
    else:
        ws = _EMPTY_F32.get(x.device)
        if ws is None:
            ws = _EMPTY_F32[x.device] = torch.empty(1, dtype=torch.float32, device=x.device)
    torch.ops.akap.dgemm(out, x, w, ws, pro, splitk, pf, residual, residual_out, ln, eps, epi,
                         ss_in, ss_out, a_out, ln_out, bn, ns, counters, bm)
    return out


def dgemm_supported(M: int, N: int, K: int, splitk: int, pf: int, epi: int = EPI_STORE,
                    bn: int = 0, inlaunch: bool = False, bm: int = 64) -> bool:
    """Mirror of dgemm_supported / gdgemm_supported / dgemm_epi_supported (host-side)."""
    if bn == 256:  # pgemm_sk: 256 x 256 tiles, any split, grid <= the CU count
        if bm != 256 or N % 256 or K % 64 or not 1 <= splitk <= 32 or K // 64 < splitk:
            return False
        return -(-M // 256) * (N // 256) * splitk <= device_cus()
    if splitk not in (1, 2, 4, 8, 16):
        return False
    if bm != 64 and not (bm == 128 and bn == 128) and not (bm == 256 and bn in (64, 128)):
        return False
    inl = inlaunch and splitk > 1 and (bn or splitk in (2, 4, 8))
    if inlaunch and splitk > 1 and not bn and splitk not in (2, 4, 8):
        return False  # the register-ring combine has 2 | 4 | 8 slices
    if epi == EPI_SILU and ((splitk != 1 and not inl) or N % 32):
        return False
    if epi == EPI_RESNORM and splitk > 1 and N % 256 and not inl:
        return False
    if bn:
        if bn not in (64, 128) or M <= 0 or N % 4 or K % splitk:
            return False
        return (K // splitk) % 64 == 0
    if M <= 0 or N <= 0 or K <= 0 or N % 4 or pf not in (1, 2, 4, 8) or K % splitk:
        return False
    return (K // splitk) % (64 * pf) == 0


_CUS: dict = {}


def device_cus(device=None) -> int:
    """Compute units of the (current) GPU; 256 (MI355X) without one."""
    key = str(device)
    if key not in _CUS:
        n = 256
        if torch.cuda.is_available():
            try:
                n = torch.cuda.get_device_properties(device or 0).multi_processor_count
            except Exception:  # pragma: no cover - device query failure
                pass
        _CUS[key] = n
    return _CUS[key]


def kgemm_supported(M: int, N: int, K: int, km: int, epi: int = EPI_STORE, pro: int = 0) -> bool:
    """Mirror of kgemm_supported (csrc/kernels/kgemm.hip)."""
    return (pro == PRO_PLAIN and km in (16, 32) and M > 0 and N % 32 == 0 and K >= 256
            and K % 256 == 0 and epi in (EPI_STORE, EPI_RESNORM))


def gdgemm_ws_floats(M: int, N: int, splitk: int, bn: int, bm: int = 64) -> int:
    """fp32 workspace of a split-K LDS-DMA GEMM (tile-padded slabs; mirrors gdgemm.hip)."""
    slabs = splitk * -(-M // bm) * -(-N // bn) * bm * bn
    return max(slabs, splitk * M * N)


_COUNTERS: dict = {}
CTR_STRIDE = 32  # ints per ticket counter: one 128-B L2 line each (csrc/kernels/common.h)
GEMM_CTR_INTS = 1 << 18  # kCtrInts
GEMM_CTR_ERR = GEMM_CTR_INTS - 1  # kCtrErr: an in-launch combine timed out


def gemm_counters(device) -> torch.Tensor:
    """Zeroed per-tile split-K tickets shared by every custom-GEMM launch on `device`
    (launches on one stream are ordered; each tile's last arriver re-arms its counter)."""
    c = _COUNTERS.get(device)
    if c is None:
        c = _COUNTERS[device] = torch.zeros(GEMM_CTR_INTS, dtype=torch.int32, device=device)
    return c


def gemm_ctr_error(device, clear: bool = True) -> int:
    """The in-launch combines' timeout flag (probe-only bn = 256 variant); host sync."""
    c = gemm_counters(device)
    v = int(c[GEMM_CTR_ERR].item())
    if clear and v:
        c[GEMM_CTR_ERR].zero_()
    return v


_EMPTY_F32: dict = {}


def gemm_splitk(M: int, N: int, K: int) -> int:
    """Split-K factor for the decode GEMM: enough 64x64 tiles x splits to cover 256 CUs,
    each split keeping >= 256 of K (mirrors gemm_splitk_choice in gemm.hip)."""
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    s = 1
    while tiles * s < 256 and K // (s * 2) >= 256:
        s *= 2
    return s


# ----------------------------------------------------------------------------- sampling
SAMPLE_MAX_CHUNKS = 64  # csrc/kernels/sampling.hip kMaxChunks
# floats per row (sample_ws_floats): 64 chunk records of 8, a 16-word filter state,
# 2 x kHistRow floats of filter-pass histograms (kHistRow = 64 x 512 float2), and the draw
# rows' tile masses (64 chunks x kMaxTiles = 64)
SAMPLE_WS_PER_ROW = SAMPLE_MAX_CHUNKS * 8 + 16 + 2 * SAMPLE_MAX_CHUNKS * 512 + SAMPLE_MAX_CHUNKS * 64
_SAMPLE_WS: dict = {}
_SAMPLE_OLD: list = []  # outgrown workspaces stay alive: captured hipGraphs address them


def _sample_ws(device, B: int):
    """Persistent sampler workspace per device: B x 64 chunk records of 32 B, B row summaries
    (M, Z, key range) for the filter kernel, and B row tickets (zeroed once; each row's last
    chunk re-arms its ticket in the kernel).  Grown, never
    shrunk: a decode hipGraph keeps the addresses it was captured with."""
    cur = _SAMPLE_WS.get(device)
    if cur is None or cur[1].numel() < B * CTR_STRIDE:
        if cur is not None:
            _SAMPLE_OLD.append(cur)
        n = max(B, 256)
        cur = (torch.zeros(n * SAMPLE_WS_PER_ROW, dtype=torch.float32, device=device),
               torch.zeros(n * CTR_STRIDE, dtype=torch.int32, device=device))
        _SAMPLE_WS[device] = cur
    return cur


def sample(logits, temperature, top_k, top_p, seeds, steps, out_tokens=None, out_logprobs=None,
           greedy_logprobs: bool = False, filtered: bool = True, greedy_only: bool = False):
    """greedy_logprobs: also return the log-prob of greedy (temperature 0) picks.  filtered=False:
    the caller guarantees no row uses top-k / top-p, so their threshold passes are skipped (the
    decode step's graph for such batches).  greedy_only: the caller guarantees every row is at
    temperature 0 and needs no log-prob -- the argmax kernel alone (out_logprobs untouched)."""
    B = logits.shape[0]
    if out_tokens is None:
        out_tokens = torch.empty(B, dtype=torch.int64, device=logits.device)
    if out_logprobs is None:
        out_logprobs = torch.empty(B, dtype=torch.float32, device=logits.device)
    if _native(logits) and greedy_only:
        torch.ops.akap.argmax(logits, out_tokens)
        return out_tokens, out_logprobs
    if _native(logits):
        ws, tickets = _sample_ws(logits.device, B)
        torch.ops.akap.sample(logits, temperature, top_k, top_p, seeds, steps, out_tokens,
                              out_logprobs, greedy_logprobs, ws, tickets, filtered)
        return out_tokens, out_logprobs
    t, lp = ref.sample(logits, temperature, top_k, top_p, seeds, steps, greedy_logprobs)
    out_tokens.copy_(t)
    out_logprobs.copy_(lp)
    return out_tokens, out_logprobs


def apply_penalties(logits, rows, toks, counts, presence, frequency, repetition):
    """In-place presence / frequency / repetition penalties on `logits` [B, V] for the
    unique (row, token, output-count) entries given in COO form."""
    if rows.numel() == 0:
        return logits
    if _native(logits):
        torch.ops.akap.apply_penalties(logits, rows, toks, counts, presence, frequency,
                                       repetition)
        return logits
    logits.copy_(ref.apply_penalties(logits, rows, toks, counts, presence, frequency,
                                     repetition))
    return logits


def argmax(logits, out=None):
    if out is None:
        out = torch.empty(logits.shape[0], dtype=torch.int64, device=logits.device)
    if _native(logits):
        torch.ops.akap.argmax(logits, out)
        return out
    out.copy_(logits.float().argmax(dim=-1))
    return out


# ----------------------------------------------------------------------------- misc
def embedding(ids, table, out=None, vocab_start: int = 0, vocab_end: Optional[int] = None):
    if vocab_end is None:
        vocab_end = vocab_start + table.shape[0]
    if out is None:
        out = torch.empty(ids.numel(), table.shape[1], dtype=table.dtype, device=table.device)
    if _native(ids):
        torch.ops.akap.embedding(ids, table, out, vocab_start, vocab_end)
        return out
    out.copy_(ref.embedding(ids, table, vocab_start, vocab_end))
    return out


def embedding_prep(ids, table, ln, residual, a_out, ss_out, zbuf, vocab_start: int = 0,
                   vocab_end: Optional[int] = None):
    """Decode prologue (csrc/kernels/embedding.hip embedding_prep_kernel): residual = the
    embedding rows, a_out = residual * ln (un-normalised), ss_out[t] = sum of squares of row t,
    zbuf zeroed -- one launch instead of embedding + RMSNorm + fill."""
    if vocab_end is None:
        vocab_end = vocab_start + table.shape[0]
    if _native(ids):
        torch.ops.akap.embedding_prep(ids, table, ln, residual, a_out, ss_out, zbuf,
                                      vocab_start, vocab_end)
        return residual, a_out, ss_out
    x = ref.embedding(ids, table, vocab_start, vocab_end)
    residual.copy_(x)
    a_out.copy_((x.float() * ln.float()).to(a_out.dtype))
    ss_out[:ids.numel()].copy_(x.float().pow(2).sum(-1))
    zbuf.zero_()
    return residual, a_out, ss_out


def moe_topk_softmax(router_logits, top_k: int, renormalize: bool = True):
    T = router_logits.shape[0]
    w = torch.empty(T, top_k, dtype=torch.float32, device=router_logits.device)
    ids = torch.empty(T, top_k, dtype=torch.int32, device=router_logits.device)
    if _native(router_logits):
        torch.ops.akap.moe_topk_softmax(router_logits, w, ids, renormalize)
        return w, ids
    rw, rid = ref.moe_topk_softmax(router_logits, top_k, renormalize)
    w.copy_(rw)
    ids.copy_(rid)
    return w, ids


def moe_router_topk(h, router, top_k: int, renormalize: bool = True):
    """Router logits (bf16, as F.linear(h, router)) -> softmax -> top-k in one launch on the
    GPU for <= 16 experts (csrc/kernels/moe.hip); the two-step path otherwise."""
    T, E = h.shape[0], router.shape[0]
    if (_native(h) and E <= 16 and T <= 2048 and h.shape[1] % 8 == 0 and h.stride(-1) == 1
            and h.stride(0) % 8 == 0):  # prefill-sized T: hipBLASLt + top-k is cheaper
        w = torch.empty(T, top_k, dtype=torch.float32, device=h.device)
        ids = torch.empty(T, top_k, dtype=torch.int32, device=h.device)
        torch.ops.akap.moe_router_topk(h, router, w, ids, renormalize)
        return w, ids
    return moe_topk_softmax(torch.nn.functional.linear(h, router), top_k, renormalize)


def moe_capacity(n: int, num_experts: int, block: int) -> int:
    cap = n + num_experts * (block - 1)
    return (cap + block - 1) // block * block


def moe_align(topk_ids, num_experts: int, block: int, inv=None, tile_expert=None):
    """Expert-sorted, block-padded index list.  Optional outputs (GPU): inv[i] = sorted
    position of flat index i; tile_expert[t] = expert of row tile t (-1 past the end)."""
    n = topk_ids.numel()
    cap = moe_capacity(n, num_experts, block)
    dev = topk_ids.device
    sorted_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    offsets = torch.empty(num_experts + 1, dtype=torch.int32, device=dev)
    num_padded = torch.empty(1, dtype=torch.int32, device=dev)
    if _native(topk_ids):
        e32 = _EMPTY_I32.get(dev)
        if e32 is None:
            e32 = _EMPTY_I32[dev] = torch.empty(0, dtype=torch.int32, device=dev)
        torch.ops.akap.moe_align(topk_ids.contiguous(), num_experts, block, sorted_ids, offsets,
                                 num_padded, e32 if inv is None else inv,
                                 e32 if tile_expert is None else tile_expert)
        return sorted_ids, offsets, num_padded
    s, o, npad = ref.moe_align(topk_ids, num_experts, block, cap)
    sorted_ids.copy_(s)
    offsets.copy_(o)
    num_padded.fill_(npad)
    return sorted_ids, offsets, num_padded


_EMPTY_I32: dict = {}
_SINK: dict = {}
MOE_BLOCK = 64


def l2_prefetch(tensors) -> None:
    """Warm the cache hierarchy with `tensors` (e.g. the next decode GEMMs' weights).
    No-op on CPU."""
    ts = [t for t in tensors if t is not None]
    if not ts or not ts[0].is_cuda:
        return
    load_native(required=True)
    dev = ts[0].device
    sink = _SINK.get(dev)
    if sink is None:
        sink = _SINK[dev] = torch.zeros(1, dtype=torch.int32, device=dev)
    for i in range(0, len(ts), 8):
        torch.ops.akap.l2_prefetch(ts[i:i + 8], sink)


def fused_moe(h, w13, w2, topk_w, topk_ids, out=None):
    """Graph-safe fused expert FFN: out[t] = sum_k w[t,k] * W2_e . silu_mul(W13_e . h[t]).

    GPU: moe_align (device-side sort + tile->expert map, 32-row tiles) -> grouped k-pipelined
    MFMA GEMM gathering token rows with the SwiGLU in its epilogue (csrc/kernels/
    moe_dgemm.hip) -> grouped GEMM -> deterministic gather-combine.  All buffer shapes depend
    only on (T, top_k, E), so the whole block captures in a hipGraph.
    w13 [E, 2F, d], w2 [E, d, F]."""
    T, d = h.shape
    K = topk_ids.shape[1]
    E = w13.shape[0]
    F = w2.shape[2]
    if out is None:
        out = torch.empty(T, d, dtype=h.dtype, device=h.device)
    if not _native(h):
        out.copy_(ref.fused_moe(h, w13, w2, topk_w, topk_ids))
        return out
    n = T * K
    bm = moe_tile_rows(n, E)
    cap = moe_capacity(n, E, bm)
    tiles = cap // bm
    dev = h.device
    inv = torch.empty(n, dtype=torch.int32, device=dev)
    tile_expert = torch.empty(tiles, dtype=torch.int32, device=dev)
    sorted_ids, _, _ = moe_align(topk_ids, E, bm, inv=inv, tile_expert=tile_expert)
    act = torch.empty(cap, F, dtype=h.dtype, device=dev)
    torch.ops.akap.moe_dgemm(act, h, w13, sorted_ids, tile_expert, n, K, True, True,
                             _moe_pf(d), bm)
    S = moe_down_splitk(n, E, bm, F)
    if S > 1:
        # fp32 K-slices of the down projection, summed by the combine (no extra launch)
        P = torch.empty(S * cap * d, dtype=torch.float32, device=dev)
        torch.ops.akap.moe_dgemm(P, act, w2, sorted_ids, tile_expert, n, K, False, False,
                                 _moe_pf(F // S), bm, S)
        torch.ops.akap.moe_combine_split(P, topk_w.contiguous(), inv, out, S, cap)
        return out
    y2 = torch.empty(cap, d, dtype=h.dtype, device=dev)
    torch.ops.akap.moe_dgemm(y2, act, w2, sorted_ids, tile_expert, n, K, False, False,
                             _moe_pf(F), bm)
    torch.ops.akap.moe_combine(y2, topk_w.contiguous(), inv, out)
    return out


def moe_down_splitk(n: int, num_experts: int, bm: int, F: int) -> int:
    """K-split of the expert down projection (K = F): with few row tiles the grid has one
    block per CU or less and each block walks all of F (measured, bench/moe_gemm_micro.py:
    Mixtral T=128 258 -> 221 us at 4 slices, T=32 271 -> 204 us at 2; none at T=256)."""
    S = 4 if (bm == 64 and n <= 40 * num_experts) else (2 if bm == 32 else 1)
    while S > 1 and (F % S or (F // S) % 64):
        S //= 2
    return S


def moe_tile_rows(n: int, num_experts: int) -> int:
    """Rows per grouped-GEMM tile: 64 once experts average more than ~20 rows (a second
    32-row tile of an expert re-streams all its weights), else 32 (less padding)."""
    return 64 if n > 20 * num_experts else 32


def _moe_pf(K: int) -> int:
    """Deepest load ring (k-tiles in flight) the reduction depth allows."""
    for pf in (4, 2, 1):
        if K % (64 * pf) == 0:
            return pf
    raise ValueError(f"MoE GEMM needs K % 64 == 0, got {K}")


def kv_gather(cache_planes, block_ids, out=None):
    planes = cache_planes.shape[0]
    blk = cache_planes[0, 0].numel()
    if out is None:
        out = torch.empty(planes, block_ids.numel(), blk, dtype=cache_planes.dtype,
                          device=cache_planes.device)
    if _native(cache_planes):
        torch.ops.akap.kv_gather(cache_planes, block_ids, out)
        return out
    out.copy_(cache_planes.reshape(planes, cache_planes.shape[1], blk)[:, block_ids.long()])
    return out


def kv_scatter(buf, cache_planes, block_ids):
    if _native(cache_planes):
        torch.ops.akap.kv_scatter(buf, cache_planes, block_ids)
        return
    planes = cache_planes.shape[0]
    blk = cache_planes[0, 0].numel()
    view = cache_planes.view(planes, cache_planes.shape[1], blk)
    view[:, block_ids.long()] = buf.view(planes, block_ids.numel(), blk)


def plane_table(planes) -> list[int]:
    """Device addresses of every plane of a cache given as [P, NB, be] plane views (one per
    allocation segment) -- the kv_pull kernel addresses planes through such a table."""
    out = []
    for pl in (planes if isinstance(planes, (list, tuple)) else [planes]):
        base, st = pl.data_ptr(), pl.stride(0) * pl.element_size()
        out += [base + i * st for i in range(pl.shape[0])]
    return out


def kv_pull(src_planes: list, src_nblocks: int, dst_planes, pairs, Hkv: int, BS: int, D: int,
            tail: Optional[torch.Tensor] = None, tail_jobs=None) -> None:
    """hipIpc KV hand-off (csrc/kernels/kv_transfer.hip): copy blocks pairs[i] = (src block,
    dst block) of every plane from the source planes (device addresses, one per plane: a
    peer's cache segments mapped by ipc_open, or this engine's own -- plane_table) into
    dst_planes ([P, NB, block_elems] views, one per segment of this engine's cache), and
    fill V tails: tail_jobs[j] = (src block, 8-token group, count 1..7, tail slot).  One
    launch on the current stream.  Every index is range-checked here, on the host, before
    anything reaches the kernel (an out-of-range block id would read or write outside the
    caches)."""
    dsts = list(dst_planes) if isinstance(dst_planes, (list, tuple)) else [dst_planes]
    nb = dsts[0].shape[1]
    be = dsts[0].shape[2]
    dst_tab = plane_table(dsts)
    if len(src_planes) != len(dst_tab):
        raise ValueError(f"kv_pull: {len(src_planes)} source planes vs {len(dst_tab)} own")
    pairs = [(int(s), int(d)) for s, d in pairs]
    for s, d in pairs:
        if not (0 <= s < src_nblocks and 0 <= d < nb):
            raise IndexError(f"kv_pull block pair ({s}, {d}) outside ({src_nblocks}, {nb})")
    jobs = [tuple(int(x) for x in j) for j in (tail_jobs or [])]
    if jobs:
        if tail is None:
            raise ValueError("tail jobs without a tail tensor")
        for s, g, c, slot in jobs:
            if not (0 <= s < src_nblocks and 0 <= g < BS // 8 and 1 <= c <= 7
                    and 0 <= slot < tail.shape[1]):
                raise IndexError(f"kv_pull tail job {(s, g, c, slot)} out of range")
    if not pairs and not jobs:
        return
    dev = dsts[0].device
    tabs = torch.tensor([list(src_planes), dst_tab], dtype=torch.int64).to(dev)
    pt = torch.tensor(pairs, dtype=torch.int32).reshape(-1).to(dev, non_blocking=True) \
        if pairs else torch.zeros(0, dtype=torch.int32, device=dev)
    jt = torch.tensor(jobs, dtype=torch.int32).reshape(-1).to(dev, non_blocking=True) \
        if jobs else None
    torch.ops.akap.kv_pull(tabs[0], tabs[1], int(be), pt, tail, jt, int(Hkv), int(BS), int(D))


def ipc_export(t: torch.Tensor) -> bytes:
    """hipIpc handle of t's allocation + t's offset in it + t's byte size (ops.cpp)."""
    load_native(required=True)
    return torch.ops.akap.ipc_export(t).numpy().tobytes()


def ipc_open(blob: bytes, device: int) -> int:
    """Map a peer's ipc_export()ed tensor; returns its device address on `device`."""
    load_native(required=True)
    return int(torch.ops.akap.ipc_open(torch.frombuffer(bytearray(blob), dtype=torch.uint8),
                                       device))


def ipc_close(addr: int) -> None:
    torch.ops.akap.ipc_close(int(addr))


def pgemm(x: torch.Tensor, w: torch.Tensor, silu: bool = False,
          offs: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None):
    """Prefill / large-M GEMM (csrc/kernels/pgemm.hip): y = x @ w.T, 256 x 256 tiles.
    silu=True: w is the [gate; up] weight [2F, K] and y = silu(x @ gate.T) * (x @ up.T) [M, F].
    offs (int32 [G] cumulative row ends): expert-grouped -- x rows sorted by group, w [G, N, K].
    The CPU path is the fp32 reference of the same op."""
    M, K = x.shape
    N = w.shape[-2]
    if out is None:
        out = torch.empty(M, N // 2 if silu else N, dtype=x.dtype, device=x.device)
    if _native(x):
        torch.ops.akap.pgemm(out, x, w, EPI_SILU if silu else EPI_STORE, offs)
        return out
    out.copy_(ref.pgemm(x, w, silu, offs))
    return out
