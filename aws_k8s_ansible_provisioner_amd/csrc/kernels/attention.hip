// Paged attention (prefill + decode) for gfx950 on MFMA 16x16x32 bf16.
//
// Design (MI355X-first, not a port of a CUDA warp kernel):
//  * One wave owns 16 "query rows".  A query row is a flattened (token, q-head of
//    the kv group) pair, so GQA heads that share a kv head share every K/V load.
//    Decode (1 token, G heads) and prefill (many tokens) run the same wave body.
//  * Scores are computed transposed, S^T = K . Q^T (rows = 16 kv tokens, cols = 16
//    query rows), so after the MFMA each lane holds 8 scores of ONE query row:
//    the online-softmax max / sum need only 2 cross-lane steps (xor 16, 32) and the
//    score registers are directly the B operand of the next MFMA.
//  * Rows of the two 16-token S tiles map to tokens 8*(r>>2) + 4*tile + (r&3), which
//    makes lane group g hold tokens 8g..8g+7 contiguous -> O^T = V^T . P^T takes V^T
//    straight from the V cache ([blk, Hkv, BS/8, D, 8]: 8-token groups, dim-major) with
//    one 16-byte load per (dim, 8 tokens), 256 contiguous bytes per 16 lanes:
//    no LDS transpose, no ds_bpermute.  O^T keeps the query row on the lane, so the
//    softmax rescale is lane-local.
//  * K operand: K cache [blk, Hkv, BS, D]; each lane loads 16 B per MFMA k-chunk.
//  * Decode: grid (seq, kv_head, partition); 4 waves split a partition's 32-token
//    chunks and combine through LDS; partitions are combined by a reduce kernel.  A wave's
//    cache block ids sit in one VGPR (read by readlane), its K/V chunks alternate between
//    two named register sets with every load unconditional (exact vmcnt counts), and in the
//    serving form the new token's K/V reach the chunk registers from LDS images, so no wave
//    waits on the prologue's cache stores (profiles/r3_attn_rework_ab.log,
//    r3_attn_fused_breakdown.log).
//  * Prefill: grid (q-tile, kv_head); each wave walks the causal range of its rows.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int kD = 128;
constexpr int kNC = kD / 32;  // MFMA k-chunks over the head dim
constexpr int kND = kD / 16;  // 16-wide dim tiles of O^T

struct WaveState {
  f32x4 o[kND];
  float m;  // running max of this lane's query row (log2 domain)
  float l;  // partial denominator (this lane's 8 tokens per chunk)
};

__device__ __forceinline__ void wave_state_init(WaveState& st) {
#pragma unroll
  for (int n = 0; n < kND; ++n) st.o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  st.m = -1e30f;
  st.l = 0.f;
}

// Register-staged operands of one 32-token KV chunk.  For an fp8 cache the raw bytes are
// staged (half the VGPRs, so the double-buffered prefetch keeps 2 waves/SIMD) and widened
// to bf16 right at the MFMA.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <bool F8>
struct ChunkT {
  bf16x8 ka[2][kNC];  // K tile rows (A operand of S^T = K . Q^T)
  bf16x8 vb[kND];     // V^T tiles (A operand of O^T = V^T . P^T)
};
template <>
struct ChunkT<true> {
  u32x2 ka[2][kNC];
  u32x2 vb[kND];
};
using ChunkRegs = ChunkT<false>;
__device__ __forceinline__ bf16x8 widen(const bf16x8& v) { return v; }
__device__ __forceinline__ bf16x8 widen(const u32x2& v) { return fp8x8_to_bf16x8(v[0], v[1]); }

template <bool F8, bool NT>
__device__ __forceinline__ auto ld_raw8(const void* base, size_t off) {
  if constexpr (F8) {
    const u32x2* p = reinterpret_cast<const u32x2*>(reinterpret_cast<const uint8_t*>(base) + off);
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
  } else {
    return ld_kv8<false, NT>(base, off);
  }
}

// Decode form: the chunk's cache block id is given (one wave-uniform value: chunks are
// 32-token aligned and BS is a multiple of 32, so a chunk never spans two blocks).  The
// decode loop keeps its block ids in a VGPR (lane j = the block of the wave's j-th chunk,
// loaded once) and reads them with readlane: an SGPR, no memory instruction in the loop.
// With a per-chunk bt[] load instead, the in-order vmcnt made every iteration wait for the
// previous chunk's K/V AND then an L2 round trip before the next chunk's loads could issue
// (the ISA showed `s_waitcnt vmcnt(2)` right after the three bt loads at the loop top).
template <bool NT = false, bool F8 = false>
__device__ __forceinline__ void load_chunk_blk(ChunkT<F8>& c, const void* __restrict__ k_cache,
                                               const void* __restrict__ v_cache, int blk,
                                               int kv_len, int kvh, int Hkv, int BS, int t0) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const int r = lane & 15;
  const size_t kb = ((size_t)blk * Hkv + kvh) * BS * kD;
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    int tok = t0 + 8 * (r >> 2) + 4 * tt + (r & 3);
    tok = min(tok, kv_len - 1);  // clamped lanes re-read a valid row (masked later)
    const size_t kp = kb + k_swz_offset(tok % BS) + 8 * g;
#pragma unroll
    for (int cc = 0; cc < kNC; ++cc) c.ka[tt][cc] = ld_raw8<F8, NT>(k_cache, kp + cc * 512);
  }
  int vt = t0 + 8 * g;
  vt = min(vt, (kv_len - 1) & ~7);
  const size_t vp = kb + ((vt % BS) >> 3) * kD * 8 + r * 8;
#pragma unroll
  for (int n = 0; n < kND; ++n) c.vb[n] = ld_raw8<F8, NT>(v_cache, vp + 16 * n * 8);
}

// Scores, online softmax and P.V for one staged chunk.
// limit: last kv position this lane's query row may attend to (-1 => none).
template <bool MASK, typename CT>
__device__ __forceinline__ void compute_chunk(WaveState& st, const bf16x8 (&qb)[kNC],
                                              const CT& c, int t0, int limit,
                                              float scale_log2) {
  const int g = (threadIdx.x & 63) >> 4;
  f32x4 s[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int cc = 0; cc < kNC; ++cc) {
    s[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(widen(c.ka[0][cc]), qb[cc], s[0], 0, 0, 0);
    s[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(widen(c.ka[1][cc]), qb[cc], s[1], 0, 0, 0);
  }
  float sv[8];
  float cmax = -INFINITY;
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float x = s[tt][i] * scale_log2;
      if (MASK) {
        const int tok = t0 + 8 * g + 4 * tt + i;
        if (tok > limit) x = -INFINITY;
      }
      sv[4 * tt + i] = x;
      cmax = fmaxf(cmax, x);
    }
  cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
  cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
  const float m_new = fmaxf(st.m, cmax);
  const float alpha = exp2f(st.m - m_new);
  st.m = m_new;
  bf16x8 pb;
  float psum = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float pj = exp2f(sv[j] - m_new);
    psum += pj;
    pb[j] = f2bf(pj);
  }
  st.l = st.l * alpha + psum;
#pragma unroll
  for (int n = 0; n < kND; ++n) {
    st.o[n] *= alpha;
    st.o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(widen(c.vb[n]), pb, st.o[n], 0, 0, 0);
  }
}

// V tail: lanes whose 8-token V group is the sequence's last group (first token gstart;
// lanes past it were clamped onto it by load_chunk) take their V^T fragments from the LDS
// group image instead of the cache.
template <bool F8>
__device__ __forceinline__ void patch_v(ChunkT<F8>& c, int t0, int gstart, const bf16* img) {
  if constexpr (!F8) {
    const int lane = threadIdx.x & 63;
    if (t0 + 8 * (lane >> 4) >= gstart) {
#pragma unroll
      for (int n = 0; n < kND; ++n)
        c.vb[n] = *reinterpret_cast<const bf16x8*>(img + (16 * n + (lane & 15)) * 8);
    }
  }
}

// The new token's K row from the LDS image the fused prologue wrote (serving path with the V
// tail): the lanes whose fragment row is token `tok` of the chunk at t0 take their 4 x 16 B
// from k_img instead of the cache, so no wave has to wait for the prologue's cache store.
template <bool F8>
__device__ __forceinline__ void patch_k(ChunkT<F8>& c, int t0, int tok, const bf16* k_img) {
  if constexpr (!F8) {
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4, r = lane & 15;
    const int pi = tok - t0;
    const bool hit = r == 4 * (pi >> 3) + (pi & 3);
    const bool t1 = (pi >> 2) & 1;
    // every lane reads the image and selects (conditional stores into one of the two tile
    // arrays made hipcc demote the chunk to scratch: 304 B/lane, 2x slower)
#pragma unroll
    for (int cc = 0; cc < kNC; ++cc) {
      const bf16x8 k8 = *reinterpret_cast<const bf16x8*>(k_img + 32 * cc + 8 * g);
      c.ka[0][cc] = hit && !t1 ? k8 : c.ka[0][cc];
      c.ka[1][cc] = hit && t1 ? k8 : c.ka[1][cc];
    }
  }
}

// Load this lane's Q^T operand for query row (lane & 15) (zeros if invalid).
__device__ __forceinline__ void load_q(bf16x8 (&qb)[kNC], const bf16* qrow_ptr, bool valid) {
  const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int c = 0; c < kNC; ++c) {
    if (valid)
      qb[c] = *reinterpret_cast<const bf16x8*>(qrow_ptr + 32 * c + 8 * g);
    else
      qb[c] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
}

// ----------------------------------------------------------------------------------
// Decode: one new token per sequence, rows = the G q-heads of one kv head.
// grid = (num_seqs, Hkv, num_parts); 4 waves split the partition's chunks.
// ----------------------------------------------------------------------------------
// Fused decode prologue: rows 0..G-1 = this kv head's G query heads, row G = its key head,
// row G+1 = its value head; 16 threads per row, 8 dims each.  q rows -> per-head RMSNorm
// (bf16-rounded, like the standalone kernel) -> NeoX RoPE -> LDS; the new token's k / v
// (only when write_kv) -> paged cache.  Rotary pairs (d, d+64) sit in threads j and j^8.
// V tail image helper: 16 threads (j = dims [8j, 8j+8)) hold an 8-token group token-major
// (rows[i] = token i) and store it as the cache's [D][8] group image (dim-major, 16 B per dim)
__device__ __forceinline__ void group_units(const bf16x8 (&rows)[8], bf16x8 (&u)[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int i = 0; i < 8; ++i) u[k][i] = rows[i][k];
}

// Fused-prologue operands loaded up front (grid decode kernel).  Every prologue load is
// issued BEFORE the first K/V chunk's loads, so the prologue's waits (counted vmcnt: the
// chunk's 16 loads were issued later) leave the chunk in flight; with the loads inside the
// prologue, their first wait drained the chunk (vmcnt is in-order) and the
// positions -> cos_sin chain added two more round trips behind it.  The V-tail rows are
// loaded whole (8 rows, valid memory) and selected afterwards: no load under a per-row
// runtime condition (hipcc would wait on each).
template <bool F8>
struct ProPre {
  bf16x8 raw, w8;
  f32x4 c0, c1, s0, s1;
  bf16x8 trow[8];
  int64_t slot;
  int tsl;
};

template <bool F8>
__device__ __forceinline__ void prologue_loads(const AttnParams& p, int seq, int kvh,
                                               int64_t pos, ProPre<F8>& pp) {
  // Branch-free: every lane loads from a valid address (lanes past the G + 2 rows re-read row
  // G + 1's bytes; a missing norm weight / tail reads the qkv row instead), so the vmcnt
  // counts stay exact -- an exec-masked branch here made hipcc wait vmcnt(0) at the merge.
  // Lanes that do not need an operand load it from one shared address (the qkv row's first
  // 16 B: one cache line per wave instruction) instead of a private one, so the branch-free
  // form costs no extra L1/L2 traffic: only the V-row lanes read the tail rows, only the q/k
  // lanes the cos/sin row and the norm weight.
  const int G = p.G;
  const int rr0 = threadIdx.x >> 4;
  const int rr = min(rr0, G + 1);
  const int j = threadIdx.x & 15;
  const bool row_lane = rr0 < G + 2, qk_lane = rr0 <= G, v_lane = rr0 == G + 1;
  const int head = rr < G ? kvh * G + rr : (rr == G ? p.Hq + kvh : p.Hq + p.Hkv + kvh);
  const bf16* row = p.qkv + (size_t)seq * p.qkv_stride;
  pp.raw = *reinterpret_cast<const bf16x8*>(row_lane ? row + head * kD + 8 * j : row);
  const bf16* nw = rr < G ? p.q_w : p.k_w;
  pp.w8 = *reinterpret_cast<const bf16x8*>(qk_lane && nw != nullptr ? nw + 8 * j : row);
  const float* cs = p.cos_sin + (size_t)pos * kD;
  const int i0 = qk_lane ? 8 * (j & 7) : 0;
  pp.c0 = *reinterpret_cast<const f32x4*>(cs + i0);
  pp.c1 = *reinterpret_cast<const f32x4*>(cs + (qk_lane ? i0 + 4 : 0));
  pp.s0 = *reinterpret_cast<const f32x4*>(cs + (qk_lane ? 64 + i0 : 0));
  pp.s1 = *reinterpret_cast<const f32x4*>(cs + (qk_lane ? 64 + i0 + 4 : 0));
  const bool tl = !F8 && p.v_tail != nullptr && v_lane;
  const bf16* tb = tl ? p.v_tail + ((size_t)max(pp.tsl, 0) * p.Hkv + kvh) * 8 * kD + 8 * j : row;
  const int ts = tl ? kD : 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) pp.trow[i] = *reinterpret_cast<const bf16x8*>(tb + (size_t)i * ts);
}

// fused_qkv_prologue on preloaded operands (same arithmetic, same stores)
// tail (the serving path: V through the V tail): the new token's K row also goes to the LDS
// image k_img and V to v_img, the chunk loop patches both in from LDS (patch_k / patch_v), so
// nothing in this kernel reads the new token's cache lines back -- the closing barrier then
// waits only for the LDS writes (lgkmcnt), not for the cache stores (with __syncthreads its
// vmcnt(0) also drained every wave's in-flight first chunk: fused 109.8 vs 105.6 us without
// the writes, profiles/r3_attn_fused_breakdown.log).
template <bool F8>
__device__ __forceinline__ void fused_qkv_prologue_pre(const AttnParams& p, int kvh,
                                                       bool write_kv, bf16* q_s, bool tail,
                                                       bf16* v_img, const ProPre<F8>& pp,
                                                       bf16* k_img) {
  const int G = p.G;
  const int rr = threadIdx.x >> 4;
  const int j = threadIdx.x & 15;
  if (rr < G + 2) {
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = bf2f(pp.raw[i]);
    if (rr <= G) {
      const bf16* nw = rr < G ? p.q_w : p.k_w;
      if (nw != nullptr) {
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) ss += x[i] * x[i];
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 16);
        const float inv = rsqrtf(ss / (float)kD + p.eps);
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = bf2f(f2bf(x[i] * inv * bf2f(pp.w8[i])));
      }
      const float cv[8] = {pp.c0[0], pp.c0[1], pp.c0[2], pp.c0[3],
                           pp.c1[0], pp.c1[1], pp.c1[2], pp.c1[3]};
      const float sv[8] = {pp.s0[0], pp.s0[1], pp.s0[2], pp.s0[3],
                           pp.s1[0], pp.s1[1], pp.s1[2], pp.s1[3]};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float other = __shfl_xor(x[i], 8, 16);
        x[i] = j < 8 ? x[i] * cv[i] - other * sv[i] : x[i] * cv[i] + other * sv[i];
      }
    }
    bf16x8 o8;
#pragma unroll
    for (int i = 0; i < 8; ++i) o8[i] = f2bf(x[i]);
    if (rr < G) {
      *reinterpret_cast<bf16x8*>(q_s + rr * kD + 8 * j) = o8;
    } else if (write_kv) {
      const int64_t slot = pp.slot;
      if (slot >= 0) {
        // tail path with defer_kv: only the LDS images here, the cache / tail stores are
        // issued at the end of the work item (deferred_kv_stores)
        const bool gst = !(tail && p.defer_kv);
        const int64_t blk = slot / p.BS;
        const int off = (int)(slot % p.BS);
        if (rr == G) {
          const size_t e = ((size_t)blk * p.Hkv + kvh) * p.BS * kD + k_swz_offset(off) +
                           k_dim_offset(8 * j);
          if constexpr (F8) {
            uint32_t* dst = reinterpret_cast<uint32_t*>((uint8_t*)p.k_cache + e);
            dst[0] = f32x4_to_fp8x4((float)o8[0], (float)o8[1], (float)o8[2], (float)o8[3]);
            dst[1] = f32x4_to_fp8x4((float)o8[4], (float)o8[5], (float)o8[6], (float)o8[7]);
          } else {
            if (gst) *reinterpret_cast<bf16x8*>((bf16*)p.k_cache + e) = o8;
            if (tail) *reinterpret_cast<bf16x8*>(k_img + 8 * j) = o8;
          }
        } else if (tail) {
          const int i0 = off & 7;
          bf16* tb = p.v_tail + ((size_t)pp.tsl * p.Hkv + kvh) * 8 * kD + 8 * j;
          bf16x8 rows[8], u[8];
#pragma unroll
          for (int i = 0; i < 8; ++i)
            rows[i] = i < i0 ? pp.trow[i] : (i == i0 ? o8 : bf16x8{0, 0, 0, 0, 0, 0, 0, 0});
          group_units(rows, u);
#pragma unroll
          for (int k = 0; k < 8; ++k) *reinterpret_cast<bf16x8*>(v_img + (8 * j + k) * 8) = u[k];
          if (!gst) {
          } else if (i0 == 7) {
            bf16* e = (bf16*)p.v_cache + ((size_t)blk * p.Hkv + kvh) * kD * p.BS +
                      (off >> 3) * kD * 8 + (size_t)(8 * j) * 8;
#pragma unroll
            for (int k = 0; k < 8; ++k) *reinterpret_cast<bf16x8*>(e + 8 * k) = u[k];
          } else {
            *reinterpret_cast<bf16x8*>(tb + (size_t)i0 * kD) = o8;
          }
        } else {
          const size_t e = ((size_t)blk * p.Hkv + kvh) * kD * p.BS + (off >> 3) * kD * 8 + (off & 7);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            if constexpr (F8)
              ((uint8_t*)p.v_cache)[e + (size_t)(8 * j + i) * 8] = f32_to_fp8((float)o8[i]);
            else
              ((bf16*)p.v_cache)[e + (size_t)(8 * j + i) * 8] = o8[i];
          }
        }
      }
    }
  }
  if (tail) {  // uniform: LDS images only; the cache stores stay in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  } else {
    __syncthreads();
  }
}

// The new token's K / V stores of the fused tail path, issued after the work item's combine
// from the LDS images the prologue built (k_img: the K row; v_img: the token's 8-token V
// group, [D][8]).  Issued in the prologue they sat in wave 0's in-order vmcnt queue ahead of
// every later chunk load, so each chunk wait of that wave also waited for the stores' write
// acknowledgements (bench/attn_fused_ab.py: fused + tail 112.7 us vs 109.4 without the stores).
// Nothing in this kernel reads those cache lines (the chunk loop patches the token in from the
// LDS images), and the next kernel sees them after the launch boundary.
template <bool F8>
__device__ __forceinline__ void deferred_kv_stores(const AttnParams& p, int kvh,
                                                   const ProPre<F8>& pp, const bf16* k_img,
                                                   const bf16* v_img) {
  const int rr = threadIdx.x >> 4;
  const int j = threadIdx.x & 15;
  const int G = p.G;
  if (rr != G && rr != G + 1) return;
  const int64_t blk = pp.slot / p.BS;
  const int off = (int)(pp.slot % p.BS);
  if (rr == G) {
    const size_t e = ((size_t)blk * p.Hkv + kvh) * p.BS * kD + k_swz_offset(off) +
                     k_dim_offset(8 * j);
    *reinterpret_cast<bf16x8*>((bf16*)p.k_cache + e) =
        *reinterpret_cast<const bf16x8*>(k_img + 8 * j);
    return;
  }
  const int i0 = off & 7;
  if (i0 == 7) {  // the group is complete: its [D][8] image goes to the cache
    bf16* e = (bf16*)p.v_cache + ((size_t)blk * p.Hkv + kvh) * kD * p.BS + (off >> 3) * kD * 8 +
              (size_t)(8 * j) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      *reinterpret_cast<bf16x8*>(e + 8 * k) =
          *reinterpret_cast<const bf16x8*>(v_img + (8 * j + k) * 8);
  } else {  // the token's row (dims 8j..8j+7) goes to the sequence's V tail
    bf16x8 o8;
#pragma unroll
    for (int i = 0; i < 8; ++i) o8[i] = v_img[(8 * j + i) * 8 + i0];
    bf16* tb = p.v_tail + ((size_t)pp.tsl * p.Hkv + kvh) * 8 * kD + 8 * j;
    *reinterpret_cast<bf16x8*>(tb + (size_t)i0 * kD) = o8;
  }
}

// Decode K/V chunks stream with non-temporal loads (read once per step; keeping them out of
// the caches leaves the L2 / MALL to the block tables, q rows and weights)
constexpr bool kDecodeNT = true;

// One (seq, kv head, partition) work item of the decode grid.
//  head: what the item needs before its first K/V byte can be requested -- the sequence's
//    length, the cache block ids of the wave's chunks (lane j: chunk pstart + 32 w + 128 j,
//    read later with readlane: an SGPR, no memory instruction in the chunk loop), in the
//    fused form the prologue's operands (ProPre, issued ahead of the chunk), then the wave's
//    first chunk in flight.  The block-id load does not wait for the length (the index is
//    clamped into the block-table row instead of guarded by it), so the chain before the
//    first K/V load is two round trips.
//  body: fused q/k-norm + RoPE + new-token K/V write (FUSED), the chunk loop over two named
//    register sets, the 4-wave LDS combine, the output (or split-KV partial) store.
template <bool FUSED, bool F8>
__device__ __forceinline__ void decode_item(const AttnParams& p, int seq, int kvh, int part,
                                            float* dyn_lds) {
  constexpr bool NT = kDecodeNT;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int g = lane >> 4;
  const int G = p.G;
  const int pstart = part * p.part_size;
  int t0 = pstart + 32 * w;
  const int tw = t0;  // the wave's first chunk (t0 itself advances in the loop below)
  const int btr =
      p.block_tables[(size_t)seq * p.bt_stride + min((t0 + 128 * lane) / p.BS, p.bt_stride - 1)];
  const int kv_len = p.seq_lens[seq];
  ProPre<F8> pp;
  if constexpr (FUSED) {  // fused-prologue operands: issued ahead of the chunk (see ProPre)
    const int64_t pos = p.positions[seq];
    pp.slot = p.slots[seq];
    pp.tsl = (!F8 && p.v_tail != nullptr) ? p.tail_slot[seq] : -1;
    prologue_loads<F8>(p, seq, kvh, pos, pp);
    __builtin_amdgcn_sched_barrier(0);
  }
  const int pend = min(kv_len, pstart + p.part_size);
  ChunkT<F8> cur;
  {
    // issued unconditionally (a wave with no chunk reads block 0, never used): a branch here
    // left the two paths with different load counts, and hipcc's merged vmcnt count then
    // waited on part of the chunk inside the prologue
    const bool has = t0 < pend;
    load_chunk_blk<NT, F8>(cur, p.k_cache, p.v_cache, has ? __builtin_amdgcn_readlane(btr, 0) : 0,
                           max(kv_len, 1), kvh, p.Hkv, p.BS, has ? t0 : 0);
  }
  const int qr = lane & 15;
  const bool valid = qr < G && kv_len > 0;
  const int q_tok = p.q_start ? p.q_start[seq] : seq;
  const bf16* qptr = FUSED ? nullptr : p.q + ((size_t)q_tok * p.Hq + kvh * G + qr) * kD;

  // combine buffer sized by G (dynamic LDS: 4 x G x (D+4) floats + stats), so small G
  // keeps LDS from limiting occupancy (G=2: ~4 KiB instead of 34 KiB)
  float* o_s = dyn_lds;                       // [4][G][kD + 4]
  float* m_s = dyn_lds + 4 * G * (kD + 4);    // [4][G]
  float* l_s = m_s + 4 * G;                   // [4][G]
#define OS(w_, r_, d_) o_s[((w_) * G + (r_)) * (kD + 4) + (d_)]
  bf16* q_s = reinterpret_cast<bf16*>(l_s + 4 * G);  // [G][kD] (fused only)
  bf16* v_img = q_s + (FUSED ? G * kD : 0);          // [kD][8] V tail group image
  bf16* k_img = v_img + kD * 8;                      // [kD] new token's K (fused + V tail)
  const int limit = kv_len - 1;
  const bool writes_kv = kv_len > 0 && pstart <= kv_len - 1 && kv_len - 1 < pend;
  // V tail: the sequence's last 8-token group (first token gstart) is read from an LDS image
  // instead of the cache -- fused: the image the prologue builds (tail + the new token);
  // plain: a still-partial group straight from the tail (the writer kernel put it there)
  int tsl;
  bool use_img;
  if constexpr (FUSED) {
    tsl = kv_len > 0 ? pp.tsl : -1;
    use_img = tsl >= 0 && writes_kv && pp.slot >= 0;
  } else {
    tsl = (!F8 && p.v_tail != nullptr && kv_len > 0) ? p.tail_slot[seq] : -1;
    use_img = tsl >= 0 && writes_kv && (kv_len & 7) != 0;
  }
  const int gstart = (kv_len - 1) & ~7;
  // j < 64 always: the host caps part_size at kDecodeMaxPart (64 chunks per wave)
  auto blk_of = [=](int tc) -> int { return __builtin_amdgcn_readlane(btr, (tc - tw) >> 7); };
  if constexpr (FUSED) {
    fused_qkv_prologue_pre<F8>(p, kvh, writes_kv, q_s, use_img, v_img, pp, k_img);
    // the chunk holding the token the prologue just wrote is re-read after the barrier (on
    // the V-tail path the loop patches it from the LDS images instead)
    if (writes_kv && !use_img && t0 < pend && t0 <= kv_len - 1 && kv_len - 1 < t0 + 32)
      load_chunk_blk<NT, F8>(cur, p.k_cache, p.v_cache, blk_of(t0), kv_len, kvh, p.Hkv, p.BS,
                             t0);
  } else if (use_img) {  // uniform per workgroup
    if (threadIdx.x < 16) {
      const int j = threadIdx.x;
      const int cnt = kv_len - gstart;
      const bf16* tb = p.v_tail + ((size_t)tsl * p.Hkv + kvh) * 8 * kD + 8 * j;
      bf16x8 rows[8], u[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        rows[i] = i < cnt ? *reinterpret_cast<const bf16x8*>(tb + (size_t)i * kD)
                          : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      group_units(rows, u);
#pragma unroll
      for (int k = 0; k < 8; ++k) *reinterpret_cast<bf16x8*>(v_img + (8 * j + k) * 8) = u[k];
    }
    __syncthreads();
  }
  WaveState st;
  wave_state_init(st);
  if (pstart < pend) {
    bf16x8 qb[kNC];
    if constexpr (FUSED) {
#pragma unroll
      for (int c = 0; c < kNC; ++c)
        qb[c] = valid ? *reinterpret_cast<const bf16x8*>(q_s + qr * kD + 32 * c + 8 * g)
                      : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    } else {
      load_q(qb, qptr, valid);
    }
    // Register double buffer as two NAMED chunk sets that alternate (the loop is unrolled by
    // two), never copied: with `cur = nxt` hipcc moved the registers at the end of each
    // iteration behind an `s_waitcnt vmcnt(0)`, so chunk i+2 could only be requested once
    // chunk i+1 had landed (one chunk in flight per wave).  Here chunk i+2's loads go into the
    // set chunk i just released while chunk i+1 may still be in flight, and each compute waits
    // only for its own set (counted vmcnt).  Loads are issued on every step: past the last
    // chunk every lane re-reads block 0's first rows (a few cache-resident lines, never used)
    // -- an `if (more)` around them made hipcc's merged vmcnt count assume the no-load path
    // and wait for the other set as well.
    ChunkT<F8> nb;
    auto fetch = [&](ChunkT<F8>& c, int tc) {
      const bool has = tc < pend;
      load_chunk_blk<NT, F8>(c, p.k_cache, p.v_cache, has ? blk_of(tc) : 0, has ? kv_len : 1,
                             kvh, p.Hkv, p.BS, has ? tc : 0);
    };
    auto consume = [&](ChunkT<F8>& c, int tc) {
      if (use_img && tc <= gstart && gstart < tc + 32) {
        patch_v(c, tc, gstart, v_img);
        if constexpr (FUSED) patch_k(c, tc, kv_len - 1, k_img);
      }
      if (tc + 31 < kv_len)
        compute_chunk<false>(st, qb, c, tc, limit, p.scale_log2);
      else
        compute_chunk<true>(st, qb, c, tc, limit, p.scale_log2);
    };
    for (; t0 < pend; t0 += 256) {
      fetch(nb, t0 + 128);
      consume(cur, t0);
      if (t0 + 128 >= pend) break;
      fetch(cur, t0 + 256);
      consume(nb, t0 + 128);
    }
  }
  float l = st.l;
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (qr < G) {
#pragma unroll
    for (int n = 0; n < kND; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) OS(w, qr, 16 * n + 4 * g + i) = st.o[n][i];
    if (g == 0) {
      m_s[w * G + qr] = st.m;
      l_s[w * G + qr] = l;
    }
  }
  __syncthreads();
  // combine: thread -> (row, 8 dims)
  const int row = threadIdx.x >> 4;
  const int d0 = (threadIdx.x & 15) * 8;
  if (row < G) {
    float M = -1e30f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, m_s[ww * G + row]);
    float L = 0.f;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float f = exp2f(m_s[ww * G + row] - M);
      L += f * l_s[ww * G + row];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f * OS(ww, row, d0 + j);
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
    if (p.num_parts == 1) {
      bf16* op = p.out + ((size_t)q_tok * p.Hq + kvh * G + row) * kD + d0;
      bf16x8 o8;
#pragma unroll
      for (int j = 0; j < 8; ++j) o8[j] = f2bf(acc[j] * inv);
      *reinterpret_cast<bf16x8*>(op) = o8;
    } else {
      const size_t pidx = ((size_t)(seq * p.Hkv + kvh) * p.num_parts + part) * G + row;
      float* po = p.part_o + pidx * kD + d0;
#pragma unroll
      for (int j = 0; j < 8; ++j) po[j] = acc[j] * inv;
      if ((threadIdx.x & 15) == 0) {
        p.part_m[pidx] = L > 0.f ? M : -1e30f;
        p.part_l[pidx] = L;
      }
    }
  }
  if constexpr (FUSED && !F8) {
    if (use_img && p.defer_kv) deferred_kv_stores<F8>(p, kvh, pp, k_img, v_img);
  }
#undef OS
}

// grid = (num_seqs, Hkv, num_parts): one work item per workgroup.  (Persistent, pipelined
// persistent, single-buffered 3-WG/CU and barrier-free-prologue forms were measured equal or
// slower and removed: profiles/r3_attn_rework_ab.log, r3_attn_variants_ab.log.)  Two
// workgroups per CU: with (256, 1) the serving form took 244 VGPRs + 32 AGPRs (one wave per
// SIMD, each CU ran its 8 workgroups of a B = 256 step one after another); bounded to two it
// fits 238 VGPRs with no spills and the next workgroup's prologue overlaps the current one's
// stream -- 110.7 -> 110.1 us serving, 106.3 -> 105.2 us on a ready q
// (profiles/r6_decode_kv_store.md).
template <bool FUSED, bool F8>
__global__ __launch_bounds__(256, 2) void paged_attn_decode_kernel(AttnParams p) {
  extern __shared__ __attribute__((aligned(16))) float dyn_lds[];
  decode_item<FUSED, F8>(p, blockIdx.x, blockIdx.y, blockIdx.z, dyn_lds);
}


// ----------------------------------------------------------------------------------
// Flash-style prefill: 128 flattened q rows (token x GQA head) per workgroup, 4 waves x 32
// rows, 64-key K/V tiles staged once per workgroup in LDS (double-buffered, next tile's
// global loads in flight during the current tile's MFMAs), v_mfma_f32_32x32x16_bf16.
//   S^T = K . Q^T : K fragments from an XOR-swizzled LDS image (A), Q^T from registers (B);
//                   each lane owns one q row (column) -> softmax is lane-local + one xor-32.
//   O^T = V^T . P^T: P^T straight from the S^T accumulators (bf16); the S^T rows are keys
//                   in fa_row_key order, so each V^T fragment is one 16-B read of the V-group
//                   image ([group][d][8 tokens], copied verbatim from the paged cache); O^T's
//                   column is again the lane's q row, so the online-softmax rescale needs no
//                   cross-lane traffic.
// ----------------------------------------------------------------------------------
// lane l <-> lane l ^ 32 reductions by one v_permlane32_swap (VALU) instead of a
// ds_bpermute round trip through LDS: with both operands = x, result [0] holds x of lanes
// 0..31 in every lane's upper-half view and [1] the other half, so op([0], [1]) is the pair's
// reduction in all 64 lanes
__device__ __forceinline__ float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x),
                                                  false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x),
                                                  false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// MFMA row r of an S^T sub-tile holds key fa_row_key(r) of the 32.  The 32x32 accumulator
// gives lane half h the rows 8 i + 4 h + (0..3); with this order its P^T fragment for k-slice
// s2 (accumulator registers 8 s2 .. 8 s2 + 7) is keys 16 s2 + 8 h + 0..7 -- one whole 8-token V
// group, so every V^T fragment is a single 16-B LDS read of the cache's group image.
__device__ __forceinline__ int fa_row_key(int r) {
  return 16 * (r >> 4) + 8 * ((r >> 2) & 1) + 4 * ((r >> 3) & 1) + (r & 3);
}

constexpr int kFaRows = 128;
constexpr int kFaKeys = 64;
constexpr int kFaBtCache = 1024;  // chunk -> block id cache in LDS (32768 keys)

__device__ __forceinline__ void fa_glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0,
                                   0);
}

// GL = true (bf16 caches): K/V tiles are staged by global_load_lds (LDS-DMA) straight into the
// next LDS buffer -- no VGPR staging registers, no ds_write pass, and the only wait for the
// next tile is the counted vmcnt at the top of the following iteration (raw s_barrier, never
// __syncthreads, whose fence would drain the DMA early).  The K image's XOR swizzle moves to
// the per-lane DMA source address (the LDS destination of a DMA is lane-linear).
// NW = waves per workgroup (4: 128 q rows, two workgroups per CU; 8: 256 q rows, one
// workgroup per CU -- every staged K/V tile feeds twice the rows).
// STAG (8 waves only): the compute/load ping-pong of the two waves that share a SIMD.  Waves
// 0-3 and 4-7 land on the same four SIMDs (one of each per SIMD) and run the same program in
// lock-step between the per-tile barriers, so both do their Q K^T MFMAs, then both their
// softmax VALU (the matrix pipe idle), then both their P V MFMAs.  With STAG the late half
// (waves 4-7) defers tile t's P V MFMAs past the next barrier: per SIMD one wave's P V(t-1)
// then Q K^T(t) run beside the other's Q K^T(t) then softmax(t) -- matrix work beside VALU
// work (MI355X_MICROARCH.md "Two waves per SIMD" item 9).  The deferred P V re-reads V(t) from
// LDS, so the ring has THREE buffers (tile t's survives until the barrier of t + 2); only the
// bf16 P fragments and the rescale factor stay in registers (+17 VGPRs).
template <bool F8, bool GL, int NW = 4, bool STAG = false>
__global__ __launch_bounds__(64 * NW, 8 / NW) void paged_attn_prefill_fa_kernel(AttnParams p) {
  constexpr int ROWS = 32 * NW;
  constexpr int NT = 64 * NW;    // threads
  constexpr int PW = 16 / NW;    // 1-KiB K (and V) DMA pieces per wave per tile
  constexpr int NBUF = STAG ? 3 : 2;
  static_assert(NW == 4 || (NW == 8 && GL), "the register-staged path assumes 256 threads");
  static_assert(!STAG || (NW == 8 && GL), "the ping-pong pairs waves w and w + 4");
  // [buf][K | V][64 keys * 128 dims] bf16 = 64 KiB (96 KiB with STAG) + the block ids of the
  // first kFaBtCache 32-key chunks; ONE __shared__ object (a second one makes hipcc drain vmcnt)
  __shared__ __attribute__((aligned(16))) bf16 lds[NBUF * 2 * kFaKeys * kD + 2 * kFaBtCache];
  int* bt_s = reinterpret_cast<int*>(lds + NBUF * 2 * kFaKeys * kD);
  // One flat grid of (tile, kv head) items, kv head innermost, dispatched back to front: the
  // host map is sorted by ascending causal work (scheduler.cpp), so every head of the longest
  // tiles starts first and the grid's tail is made of the shortest ones (longest-first over
  // the whole grid, not per head: a (tile, head) grid put all of head 7's long tiles last).
  // With Hkv = 8 the dispatcher's round-robin over the 8 XCDs keeps one head's tiles -- which
  // read the same K/V -- on one XCD's L2.
  const int flat = gridDim.x - 1 - blockIdx.x;
  const int tile = flat / p.Hkv;
  const int kvh = flat - tile * p.Hkv;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar registers
  const int r = lane & 31;
  const int h = lane >> 5;
  const int seq = __builtin_amdgcn_readfirstlane(p.tile_seq[tile]);  // scalar: bt is uniform
  const int q0 = p.q_start[seq];
  const int q_len = p.q_start[seq + 1] - q0;
  const int kv_len = p.seq_lens[seq];
  const int G = p.G;
  const int row0 = p.tile_row[tile];
  const int R = row0 + 32 * w + r;
  const int pos = R / G;
  const int hig = R % G;
  const bool valid = pos < q_len;
  const int ctx0 = kv_len - q_len;  // keys before this chunk's first query token
  const int limit = valid ? ctx0 + pos : -1;

  // Q^T fragments (B operand): lane (r, h) holds Q[row][16 s + 8 h + j].  Loaded after the
  // first K/V tile's DMA is issued, so the q round trips (and the fused q prep) overlap it.
  bf16x8 qf[8];
  auto load_q = [&]() {
  if (p.qkv != nullptr) {
    // fused q prep (the standalone qk_norm_rope_cache pass then skips these tokens' q heads):
    // the raw q row straight from the QKV projection, per-head RMSNorm over the lane pair
    // (r, r + 32) that holds its 128 dims (one v_permlane32_swap), bf16-rounded like the
    // standalone kernel, then NeoX rotary -- dims d < 64 (s8 < 4) pair with d + 64 (s8 + 4)
    // in the same lane, so the rotation is lane-local.  Same arithmetic as rope_cache.hip
    // qk_tok.
    const int tok = q0 + (valid ? pos : 0);
    const bf16* src = p.qkv + (size_t)tok * p.qkv_stride + (size_t)(kvh * G + hig) * kD + 8 * h;
    // rotary position = the token's key index ctx0 + pos -- the invariant the causal limit
    // above already relies on (positions[tok] holds the same value): no dependent load
    const float* cs = p.cos_sin + (size_t)(valid ? ctx0 + pos : 0) * kD + 8 * h;
    // every operand load issued up front, unconditionally (one round trip; without a q norm
    // the weight loads read valid rotary-table bytes and are ignored)
    const bool qn = p.q_w != nullptr;
    const bf16* wsrc = qn ? p.q_w : reinterpret_cast<const bf16*>(p.cos_sin);
    bf16x8 raw[8], w8[8];
    f32x4 cv[4][2], sv[4][2];
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) raw[s8] = *reinterpret_cast<const bf16x8*>(src + 16 * s8);
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {
      // both 8-dim halves at wave-uniform addresses (scalar loads: 512 B per wave instead of
      // 8 KB of vector loads of the same 256-B weight row), then the lane's half selected
      typedef const __attribute__((address_space(4))) bf16x8 cbf16x8;  // constant: s_load
      const bf16x8 wl = *(cbf16x8*)(size_t)(wsrc + 16 * s8);
      const bf16x8 wh = *(cbf16x8*)(size_t)(wsrc + 16 * s8 + 8);
      w8[s8] = h ? wh : wl;
    }
#pragma unroll
    for (int s8 = 0; s8 < 4; ++s8)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        cv[s8][k] = *reinterpret_cast<const f32x4*>(cs + 16 * s8 + 4 * k);
        sv[s8][k] = *reinterpret_cast<const f32x4*>(cs + 64 + 16 * s8 + 4 * k);
      }
    float ss = 0.f;
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8)
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += bf2f(raw[s8][j]) * bf2f(raw[s8][j]);
    const float inv = rsqrtf(xor32_sum(ss) / (float)kD + p.eps);
    // normed value of dim (s8, j), bf16-rounded like the standalone kernel (raw without a norm)
    auto xn = [&](int s8, int j) {
      const float v = bf2f(raw[s8][j]);
      return qn ? bf2f(f2bf(v * inv * bf2f(w8[s8][j]))) : v;
    };
#pragma unroll
    for (int s8 = 0; s8 < 4; ++s8) {
      bf16x8 lo, hi;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c = cv[s8][j >> 2][j & 3], sn = sv[s8][j >> 2][j & 3];
        const float x1 = xn(s8, j), x2 = xn(s8 + 4, j);
        lo[j] = f2bf(x1 * c + -1.f * x2 * sn);
        hi[j] = f2bf(x2 * c + 1.f * x1 * sn);
      }
      const bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      qf[s8] = valid ? lo : z;
      qf[s8 + 4] = valid ? hi : z;
    }
  } else {
    const bf16* qrow = p.q + ((size_t)(q0 + (valid ? pos : 0)) * p.Hq + kvh * G + hig) * kD;
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8)
      qf[s8] = valid ? *reinterpret_cast<const bf16x8*>(qrow + 16 * s8 + 8 * h)
                     : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  };

  const int wg_last_pos = min(q_len - 1, (row0 + ROWS - 1) / G);
  const int wg_limit = ctx0 + wg_last_pos;
  const int ntiles = wg_limit / kFaKeys + 1;
  const int w_first_pos = (row0 + 32 * w) / G;
  const int w_last_pos = min(q_len - 1, (row0 + 32 * w + 31) / G);
  const bool wave_active = w_first_pos < q_len;
  const int w_limit = ctx0 + w_last_pos;       // last key any row of this wave sees
  const int w_min_limit = ctx0 + w_first_pos;  // every row of this wave sees keys <= this
  const int* bt = p.block_tables + (size_t)seq * p.bt_stride;
  const int BS = p.BS;
  const int last_chunk = (kv_len - 1) >> 5;

  // staging: 1024 16-B pieces of K and 1024 of V per tile, 4 + 4 per thread
  bf16x8 kst[4], vst[4];
  auto stage_load = [&](int t) {
    // block ids first (LDS), then all 8 global loads back to back: no wait between them
    int blk[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = (tid + 256 * i) >> 9;
      blk[i] = bt_s[min(t * 2 + c, last_chunk)];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pc = tid + 256 * i;   // 0..1023
      const int c = pc >> 9;           // 32-key chunk of the tile
      const int within = pc & 511;
      const int off = (min(t * 2 + c, last_chunk) * 32) % BS;
      const size_t base = ((size_t)blk[i] * p.Hkv + kvh) * BS * kD + (size_t)off * kD;
      // fp8 caches: 8-byte loads widened to bf16 here, so the LDS images are the same
      kst[i] = ld_kv8<F8, false>(p.k_cache, base + within * 8);
      vst[i] = ld_kv8<F8, false>(p.v_cache, base + within * 8);
    }
  };
  auto stage_store = [&](int buf) {
    bf16* kl = lds + (size_t)buf * 2 * kFaKeys * kD;
    bf16* vl = kl + kFaKeys * kD;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pc = tid + 256 * i;
      const int c = pc >> 9;
      const int within = pc & 511;
      // K cache chunk order: ((tt * 4 + cc) * 16 + r16) * 4 + q  (16-B pieces)
      const int q4 = within & 3;
      const int r16 = (within >> 2) & 15;
      const int cc = (within >> 6) & 3;
      const int tt = within >> 8;
      const int key = 32 * c + 8 * (r16 >> 2) + 4 * tt + (r16 & 3);
      const int dc = 4 * cc + q4;  // 16-B column of the 256-B key row
      *reinterpret_cast<bf16x8*>(kl + key * kD + ((dc ^ (key & 15)) * 8)) = kst[i];
      *reinterpret_cast<bf16x8*>(vl + c * 32 * kD + within * 8) = vst[i];
    }
  };

  // LDS-DMA staging of tile t into buffer buf: 16 K + 16 V instructions of 1 KiB, 4 + 4 per
  // wave.  K: LDS 16-B slot s holds (key s/16, logical column (s%16) ^ (key&15)); the lane
  // writing slot s loads that piece from the fragment-ordered K cache chunk.  Every piece a
  // wave stages lies in 32-key chunk (w >> 1) of the tile, so the chunk base is wave-uniform
  // (scalar) and the per-lane offsets are the same for every tile.
  int koff[PW], voff[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int s = (w * PW + i) * 64 + lane;
    const int key = s >> 4;
    const int dc = (s & 15) ^ (key & 15);
    const int k32 = key & 31;
    const int tt = (k32 >> 2) & 1, r16 = ((k32 >> 3) << 2) | (k32 & 3);
    koff[i] = (((tt * 4 + (dc >> 2)) * 16 + r16) * 4 + (dc & 3)) * 8;
    voff[i] = (s & 511) * 8;
  }
  // wave-uniform chunk -> its block id by a scalar load straight from the block table (no LDS
  // copy of the table, no workgroup barrier before the first DMA); loaded one tile ahead of
  // its DMA, so the load is retired by the next iteration's lgkmcnt wait
  auto chunk_of = [&](int t) {
    return __builtin_amdgcn_readfirstlane(min(t * 2 + ((w * PW) >> 3), last_chunk));
  };
  // through the constant address space: a uniform load from it is a scalar (s_load) read of
  // the block table, which this kernel never writes
  const __attribute__((address_space(4))) int* bt_c =
      (const __attribute__((address_space(4))) int*)bt;
  auto blk_of = [&](int t) { return bt_c[chunk_of(t) * 32 / BS]; };
  auto stage_glds = [&](int t, int buf, int blk) {
    bf16* kl = lds + (size_t)buf * 2 * kFaKeys * kD;
    bf16* vl = kl + kFaKeys * kD;
    const int chunk = chunk_of(t);
    const size_t base =
        ((size_t)blk * p.Hkv + kvh) * BS * kD + (size_t)((chunk * 32) % BS) * kD;
    const bf16* kb = static_cast<const bf16*>(p.k_cache) + base;
    const bf16* vb = static_cast<const bf16*>(p.v_cache) + base;
#pragma unroll
    for (int i = 0; i < PW; ++i) fa_glds16(kb + koff[i], kl + (w * PW + i) * 512);
#pragma unroll
    for (int i = 0; i < PW; ++i) fa_glds16(vb + voff[i], vl + (w * PW + i) * 512);
  };

  int blk_next = 0;
  if constexpr (GL) {
    stage_glds(0, 0, blk_of(0));
    blk_next = blk_of(1);
    load_q();
  } else {
    load_q();
    // register-staged form: per-piece block ids come from an LDS copy of the table
    for (int c = tid; c <= last_chunk; c += NT) bt_s[c] = bt[c * 32 / BS];
    __syncthreads();
    stage_load(0);
    stage_store(0);
    __syncthreads();
  }
  // accumulators zeroed after the prologue (not live across the q loads / q prep)
  f32x16 oacc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) oacc[i][j] = 0.f;
  float m_run = -1e30f, l_run = 0.f;
  // STAG, late waves: tile t-1's P fragments and rescale, applied after the next barrier
  bf16x8 pd[2][2];
  float alpha_d = 1.f;
  bool resc_d = false, pend = false;
  // the deferred O^T += V^T P^T of tile tp (its V still in LDS buffer tp % NBUF)
  auto deferred_pv = [&](int tp) {
    if (resc_d) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) oacc[i][j] *= alpha_d;
    }
    const bf16* vlp = lds + (size_t)(tp % NBUF) * 2 * kFaKeys * kD + kFaKeys * kD;
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 v4[4];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          v4[dt] = *reinterpret_cast<const bf16x8*>(vlp + ((4 * k + 2 * s2 + h) * kD + 32 * dt + r) * 8);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          oacc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v4[dt], pd[k][s2], oacc[dt], 0, 0, 0);
      }
    pend = false;
  };
  // the K/V loop, instantiated once per wave role: the early and late STAG paths keep
  // different registers live across the barrier, so one runtime-branching loop would have to
  // hold both sets (it spilled); two loops let each keep only its own
  auto kv_loop = [&](auto late_c) {
  constexpr bool late = decltype(late_c)::value;
  for (int t = 0; t < ntiles; ++t) {
    const int buf = STAG ? t % NBUF : (t & 1);
    const bool more = t + 1 < ntiles;
    if constexpr (GL) {
      // tile t (issued one iteration ago) landed for this wave; every wave's LDS reads of
      // the buffer tile t+1 goes into (tile t-1, or t-2 with STAG) are done -> after the
      // barrier it may be refilled
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (more) {
        stage_glds(t + 1, STAG ? (t + 1) % NBUF : (buf ^ 1), blk_next);
        blk_next = blk_of(t + 2);
      }
    } else {
      if (more) stage_load(t + 1);
    }
    if (late && pend) deferred_pv(t - 1);
    const int key0 = t * kFaKeys;
    if (wave_active && key0 <= w_limit) {
      const bf16* kl = lds + (size_t)buf * 2 * kFaKeys * kD;
      const bf16* vl = kl + kFaKeys * kD;
      // S^T = K . Q^T for the two 32-key sub-tiles (interleaved: independent chains)
      f32x16 sacc[2];
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int j = 0; j < 16; ++j) sacc[k][j] = 0.f;
      // every K fragment of the tile is requested before the first MFMA, so the LDS latency
      // is paid once per tile, not once per MFMA
      bf16x8 kf[8][2];
#pragma unroll
      for (int s8 = 0; s8 < 8; ++s8)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int key = 32 * k + fa_row_key(r);
          kf[s8][k] = *reinterpret_cast<const bf16x8*>(
              kl + key * kD + (((2 * s8 + h) ^ (key & 15)) * 8));
        }
#pragma unroll
      for (int s8 = 0; s8 < 8; ++s8)
#pragma unroll
        for (int k = 0; k < 2; ++k)
          sacc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[s8][k], qf[s8], sacc[k], 0, 0, 0);
      // likewise the V^T fragments: requested now, their latency hides under the softmax
      // (late STAG waves re-read them when their deferred P V runs)
      bf16x8 vf[2][2][4];
      if (!late) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
              vf[k][s2][dt] = *reinterpret_cast<const bf16x8*>(
                  vl + ((4 * k + 2 * s2 + h) * kD + 32 * dt + r) * 8);
      }
      // causal mask (wave-uniform branch: only tiles that cross this wave's diagonal pay for
      // it) and the running max on the raw scores -- the log2-domain scale is positive, so
      // it commutes with max and folds into the exponent's FMA below
      const bool need_mask = key0 + kFaKeys - 1 > w_min_limit;
      float mx = -INFINITY;
      if (need_mask) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int kk = key0 + 32 * k + 16 * (j >> 3) + 8 * h + (j & 7);
            if (kk > limit) sacc[k][j] = -INFINITY;
            mx = fmaxf(mx, sacc[k][j]);
          }
      } else {
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int j = 0; j < 16; ++j) mx = fmaxf(mx, sacc[k][j]);
      }
      mx = xor32_max(mx);
      // deferred max: the running max (and with it every rescale of O and l) moves only when
      // the tile's max exceeds it by more than rescale_t log2 units -- P entries then reach at
      // most 2^rescale_t, exact in the fp32 sums and as relative-precision bf16 P.  With one
      // branch per wave (__any below) an exact running max rescaled almost every tile: some
      // of the wave's 32 rows nearly always sees a new maximum.
      const float m_cand = fmaxf(m_run, mx * p.scale_log2);
      const float m_new = m_cand > m_run + p.rescale_t ? m_cand : m_run;
      // raw v_exp_f32 (no denormal range fix-up: arguments are <= 0, tiny results flush)
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      float rsp[4] = {0.f, 0.f, 0.f, 0.f};  // four short add chains instead of one of 32
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const float e = __builtin_amdgcn_exp2f(fmaf(sacc[k][j], p.scale_log2, -m_new));
          sacc[k][j] = e;
          rsp[j & 3] += e;
        }
      const float rs = xor32_sum((rsp[0] + rsp[1]) + (rsp[2] + rsp[3]));
      l_run = l_run * alpha + rs;
      if (late) {  // P V of this tile after the next barrier (deferred_pv)
        resc_d = __any(m_new != m_run);
        alpha_d = alpha;
        m_run = m_new;
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int j = 0; j < 8; ++j) pd[k][s2][j] = f2bf(sacc[k][8 * s2 + j]);
        pend = true;
        continue;
      }
      // rescale only when some row's running max moved (alpha == 1 exactly otherwise): past
      // the first tiles of a causal row the max rarely changes
      if (__any(m_new != m_run)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 16; ++j) oacc[i][j] *= alpha;
      }
      m_run = m_new;
      // O^T += V^T . P^T: P^T from the S^T accumulators; V^T fragments loaded per (k, s2)
      // pair ahead of their 4 independent (per d-tile) MFMAs
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 pb;
#pragma unroll
          for (int j = 0; j < 8; ++j) pb[j] = f2bf(sacc[k][8 * s2 + j]);
          // keys 16 s2 + 8 h + 0..7 of sub-tile k = V group 4 k + 2 s2 + h (vf above)
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
            oacc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[k][s2][dt], pb, oacc[dt], 0,
                                                               0, 0);
        }
    }
    if constexpr (!GL) {
      if (more) stage_store(buf ^ 1);
      __syncthreads();
    }
  }
  if (late && pend) deferred_pv(ntiles - 1);
  };
  if constexpr (STAG) {
    if (w >= 4) kv_loop(std::true_type{});
    else kv_loop(std::false_type{});
  } else {
    kv_loop(std::false_type{});
  }
  // O^T accumulator of lane (r, h): row r's dims 32 dt + 8 j4 + 4 h + (0..3).  Each pair of
  // 8-dim groups (j4 = 2 kp, 2 kp + 1) is exchanged between the lane halves with two
  // v_permlane32_swap, after which lane r holds dims 16 kp + 0..7 and lane r + 32 dims
  // 16 kp + 8..15 of the same row: one 16-B store per pair instead of two 8-B stores (the
  // epilogue is store-issue bound: 18 us of 117 at 32 x 512, profiles/r2_pmc_prefill_v2.md)
  const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
  bf16* orow = p.out + ((size_t)(q0 + (valid ? pos : 0)) * p.Hq + kvh * G + hig) * kD;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int kp = 0; kp < 2; ++kp) {
      bf16x4 oa, ob;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        oa[i] = f2bf(oacc[dt][8 * kp + i] * inv);
        ob[i] = f2bf(oacc[dt][8 * kp + 4 + i] * inv);
      }
      const u32x2 a = __builtin_bit_cast(u32x2, oa), b = __builtin_bit_cast(u32x2, ob);
      const auto r0 = __builtin_amdgcn_permlane32_swap(a[0], b[0], false, false);
      const auto r1 = __builtin_amdgcn_permlane32_swap(a[1], b[1], false, false);
      const u32x4 o = {r0[0], r1[0], r0[1], r1[1]};
      // every lane takes part in the swaps; only rows of this chunk store
      if (valid) *reinterpret_cast<u32x4*>(orow + 32 * dt + 16 * kp + 8 * h) = o;
    }
}

// Combine split-KV partitions: grid (num_seqs, Hkv), 256 threads = (16 rows x 16 lanes x 8 dims).
__global__ __launch_bounds__(256) void paged_attn_reduce_kernel(AttnParams p) {
  const int seq = blockIdx.x;
  const int kvh = blockIdx.y;
  const int G = p.G;
  const int row = threadIdx.x >> 4;
  const int d0 = (threadIdx.x & 15) * 8;
  if (row >= G) return;
  const int kv_len = p.seq_lens[seq];
  const int nparts = min(p.num_parts, (kv_len + p.part_size - 1) / p.part_size);
  const size_t base = ((size_t)(seq * p.Hkv + kvh) * p.num_parts) * G + row;
  float M = -1e30f;
  for (int q = 0; q < nparts; ++q) M = fmaxf(M, p.part_m[base + (size_t)q * G]);
  float L = 0.f;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int q = 0; q < nparts; ++q) {
    const size_t idx = base + (size_t)q * G;
    const float f = exp2f(p.part_m[idx] - M) * p.part_l[idx];
    L += f;
    const f32x4* po = reinterpret_cast<const f32x4*>(p.part_o + idx * kD + d0);
    f32x4 a = po[0], b = po[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] += f * a[j];
      acc[4 + j] += f * b[j];
    }
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  const int q_tok = p.q_start ? p.q_start[seq] : seq;
  bf16* op = p.out + ((size_t)q_tok * p.Hq + kvh * G + row) * kD + d0;
  bf16x8 o8;
#pragma unroll
  for (int j = 0; j < 8; ++j) o8[j] = f2bf(acc[j] * inv);
  *reinterpret_cast<bf16x8*>(op) = o8;
}

void launch_paged_attn_prefill(const AttnParams& p, int num_tiles, int tile_rows,
                               hipStream_t s) {
  if (num_tiles == 0) return;
  const dim3 grid(num_tiles * p.Hkv);  // flat (tile, kv head), see the kernel
  static const float rescale_t = [] {  // AKAP_FA_RESCALE_T (log2 units; 0 = exact max)
    const char* e = std::getenv("AKAP_FA_RESCALE_T");
    return e != nullptr ? (float)std::atof(e) : 8.f;
  }();
  AttnParams q = p;
  q.rescale_t = rescale_t;
  // AKAP_PREFILL_STAGGER=1: the 8-wave kernel's compute/load ping-pong (STAG above)
  static const bool stag = [] {
    const char* e = std::getenv("AKAP_PREFILL_STAGGER");
    return e != nullptr && std::atoi(e) == 1;
  }();
  if (tile_rows == 2 * kFaRows && !p.kv_fp8) {  // 256 rows, 8 waves (bf16 caches)
    if (stag) paged_attn_prefill_fa_kernel<false, true, 8, true><<<grid, 512, 0, s>>>(q);
    else paged_attn_prefill_fa_kernel<false, true, 8><<<grid, 512, 0, s>>>(q);
  }
  else if (p.kv_fp8)  // fp8 caches: register-staged (widened to bf16 on the way into LDS)
    paged_attn_prefill_fa_kernel<true, false><<<grid, 256, 0, s>>>(q);
  else  // bf16 caches: LDS-DMA staging
    paged_attn_prefill_fa_kernel<false, true><<<grid, 256, 0, s>>>(q);
}

void launch_paged_attn_decode(const AttnParams& p, int num_seqs, hipStream_t s) {
  if (num_seqs == 0) return;
  const size_t smem = (size_t)(4 * p.G * (kD + 4) + 8 * p.G) * sizeof(float) +
                      (p.qkv ? (size_t)p.G * kD * sizeof(bf16) : 0) +
                      (p.v_tail ? (size_t)kD * 8 * sizeof(bf16) : 0) +
                      (p.qkv && p.v_tail ? (size_t)kD * sizeof(bf16) : 0);
  const dim3 grid(num_seqs, p.Hkv, p.num_parts);
  static const int defer_kv = [] {  // AKAP_DECODE_DEFER_KV=0: stores in the prologue (A/B)
    const char* e = std::getenv("AKAP_DECODE_DEFER_KV");
    return e != nullptr ? std::atoi(e) : 1;
  }();
  AttnParams q = p;
  q.defer_kv = defer_kv;
  if (p.kv_fp8) {
    if (p.qkv != nullptr) paged_attn_decode_kernel<true, true><<<grid, 256, smem, s>>>(q);
    else paged_attn_decode_kernel<false, true><<<grid, 256, smem, s>>>(q);
  } else {
    if (p.qkv != nullptr) paged_attn_decode_kernel<true, false><<<grid, 256, smem, s>>>(q);
    else paged_attn_decode_kernel<false, false><<<grid, 256, smem, s>>>(q);
  }
  if (p.num_parts > 1) paged_attn_reduce_kernel<<<dim3(num_seqs, p.Hkv), 256, 0, s>>>(q);
}

}  // namespace akap
