// Fused post-QKV-projection epilogue for gfx950:
//   per-head RMSNorm on q and k (Qwen3; optional)  ->  NeoX rotary on q and k
//   -> q written contiguous [T, Hq, D]; k, v scattered into the paged KV cache.
//
// One pass over the QKV activations instead of three (norm, rope, cache write), one
// launch: q/k heads and V spans are distinct workgroup roles of the same grid.  cos/sin come
// from a host-precomputed fp32 table [max_pos, D] (cos | sin), no on-device trig.
//
// Paged cache layouts (MI355X-first, chosen so the attention kernels can issue
// 16-byte MFMA-operand loads with no transpose, 1 KiB contiguous per load instruction):
//   K cache: [num_blocks, Hkv, BS, D] shape, MFMA-fragment order inside each 32-token
//            chunk (k_swz_offset in common.h)
//   V cache: [num_blocks, Hkv, BS/8, D, 8] (8-token groups, dim-major inside a group):
//            the attention kernel's V^T operand (one dim, 8 consecutive tokens) is one
//            16-byte load, and a token's 128 dims land in 16-byte-strided slots of one
//            2 KiB group (4x fewer cache lines touched per written token than [D][BS]).
#include "common.h"
#include "kernels.h"

namespace akap {

// q/k role: 16 lanes own one token; lane i holds the 8 contiguous dims [8i, 8i+8) of a head
// row (one 16-byte load / store), its rotate-half partner dims live in lane i ^ 8 and are
// fetched with one DPP row-rotate per packed pair.  The K row goes to the cache as 16-byte
// stores (8 dims never straddle a 32-dim fragment group).
__device__ __forceinline__ uint32_t dpp_xor8(uint32_t v) {
  // row_ror:8 inside a 16-lane DPP row == lane ^ 8
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false);
}

// Sum over a 16-lane DPP row (the lanes of one token), on VALU lane swaps: xor 1 and 2 as
// quad permutes, then the half-row and row mirrors (each leaves 4-, 8-, 16-lane groups
// uniform) -- no ds_bpermute round trips.
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xf, 0xf, false));
  return v;
}

// q/k role, token-major: 16 lanes own one token and walk its Hq + Hkv heads, 8 head rows'
// loads in flight at a time (index clamped, so every load is unconditional); the token's
// position, slot, rotary row and the two norm weights are read once per token instead of
// once per (token, head) -- with one item per (token, head) the dependent position -> rotary
// loads and the short-lived workgroups left the kernel latency-bound (~3.8 TB/s at 16k tokens).
template <bool F8>
__device__ __forceinline__ void qk_tok(const bf16* __restrict__ qkv, int qkv_stride,
                                       bf16* __restrict__ q_out, void* __restrict__ k_cache,
                                       const int64_t* __restrict__ positions,
                                       const int64_t* __restrict__ slots,
                                       const float* __restrict__ cos_sin,
                                       const bf16* __restrict__ q_w, const bf16* __restrict__ k_w,
                                       int T, int Hq, int Hkv, int BS, float eps, int apply_rope,
                                       int q_rows) {
  constexpr int D = 128, HALF = 64, HB = 8;
  const int t = blockIdx.x * 16 + (threadIdx.x >> 4);
  const int li = threadIdx.x & 15;
  // every lane of a 16-lane row shares the token, so rows exit together (DPP stays valid)
  if (t >= T) return;
  const int H = Hq + Hkv;
  f32x4 c0 = {1.f, 1.f, 1.f, 1.f}, c1 = c0, s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
  if (apply_rope) {
    const float* cs = cos_sin + (size_t)positions[t] * D + 8 * (li & 7);
    c0 = *reinterpret_cast<const f32x4*>(cs);
    c1 = *reinterpret_cast<const f32x4*>(cs + 4);
    s0 = *reinterpret_cast<const f32x4*>(cs + HALF);
    s1 = *reinterpret_cast<const f32x4*>(cs + HALF + 4);
  }
  const int64_t slot = slots[t];
  const bf16x8 zero8 = {};
  const bf16x8 qw8 = q_w ? *reinterpret_cast<const bf16x8*>(q_w + 8 * li) : zero8;
  const bf16x8 kw8 = k_w ? *reinterpret_cast<const bf16x8*>(k_w + 8 * li) : zero8;
  const float sg = li < 8 ? -1.f : 1.f;  // first half: x1 c - x2 s; second: x2 c + x1 s
  const bf16* row = qkv + (size_t)t * qkv_stride + 8 * li;
  // tokens at or past q_rows (>= 0) take only their k heads: their q rows are normed and
  // rotated by the prefill attention kernel itself, straight from the QKV rows
  const int hstart = (q_rows < 0 || t < q_rows) ? 0 : Hq;
  for (int h0 = hstart; h0 < H; h0 += HB) {
    bf16x8 raw[HB];
#pragma unroll
    for (int j = 0; j < HB; ++j) raw[j] = *reinterpret_cast<const bf16x8*>(row + min(h0 + j, H - 1) * D);
#pragma unroll
    for (int j = 0; j < HB; ++j) {
      const int h = h0 + j;
      if (h >= H) break;  // uniform
      const bool is_q = h < Hq;
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = bf2f(raw[j][e]);
      if (is_q ? q_w != nullptr : k_w != nullptr) {
        float ss = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) ss += x[e] * x[e];
        const float inv = rsqrtf(row16_sum(ss) / (float)D + eps);
        const bf16x8 w = is_q ? qw8 : kw8;
        // round-trip through bf16 like the reference module (norm output is bf16)
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = bf2f(f2bf(x[e] * inv * bf2f(w[e])));
      }
      if (apply_rope) {
        // partner values are exactly representable in bf16 here (raw input or bf16-rounded
        // norm output), so they travel packed: 4 DPP moves for 8 values
        uint32_t pp[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bf16x2 v2 = {f2bf(x[2 * e]), f2bf(x[2 * e + 1])};
          pp[e] = dpp_xor8(__builtin_bit_cast(uint32_t, v2));
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bf16x2 p2 = __builtin_bit_cast(bf16x2, pp[e >> 1]);
          const float pv = bf2f(p2[e & 1]);
          const float c = e < 4 ? c0[e] : c1[e - 4];
          const float sn = e < 4 ? s0[e] : s1[e - 4];
          x[e] = x[e] * c + sg * pv * sn;
        }
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(x[e]);
      if (is_q) {
        *reinterpret_cast<bf16x8*>(q_out + ((size_t)t * Hq + h) * D + 8 * li) = o;
      } else if (slot >= 0) {
        const int64_t blk = slot / BS;
        const int off = (int)(slot % BS);
        const size_t e = ((size_t)blk * Hkv + (h - Hq)) * BS * D + k_swz_offset(off) +
                         k_dim_offset(8 * li);
        if constexpr (F8) {
          // from the bf16-rounded values (same rounding chain as the bf16 cache + reference)
          typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
          u32x2 wv;
          wv[0] = f32x4_to_fp8x4((float)o[0], (float)o[1], (float)o[2], (float)o[3]);
          wv[1] = f32x4_to_fp8x4((float)o[4], (float)o[5], (float)o[6], (float)o[7]);
          *reinterpret_cast<u32x2*>(reinterpret_cast<uint8_t*>(k_cache) + e) = wv;
        } else {
          *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(k_cache) + e) = o;
        }
      }
    }
  }
}

// v role: one workgroup per (64-token span of the batch, kv head).  V rows are staged
// through LDS with 16-byte loads; each run of batch tokens that falls into one 8-token
// slot group (its "leader" is the run's first token) is written by the span holding the
// leader: a complete group as one 16-byte [D][8] vector per dim, a partial group (chunk
// edges, decode tokens) as 2-byte scatters.  Written slots are never shared between
// sequences (shared prefix blocks are full and read-only), so a run of consecutive slots
// is one sequence's consecutive positions.
constexpr int V_SPAN = 64;
constexpr int V_ROWS = V_SPAN + 7;  // a run starting in the span may end 7 tokens past it

//
// Every global read of the role is issued before the first is consumed: the span's V rows
// (5 unconditional, index-clamped 16-byte loads per thread) and its slots (slots[t0 - 1 ..
// t0 + V_ROWS), one per thread) land in registers, then in LDS, and the run scan reads the
// slots from LDS.  A strided fill loop and a scan of slots[] in global memory made the role a
// chain of ~5 + 8 dependent round trips per workgroup (round 6: 44 us per 16k-token prefill
// layer in the serving trace, ~3 TB/s of K/V traffic).
template <bool F8>
__device__ __forceinline__ void v_span(const bf16* __restrict__ qkv, int qkv_stride,
                                       void* __restrict__ v_cache,
                                       const int64_t* __restrict__ slots, int T, int Hq, int Hkv,
                                       int BS, int span_id, bf16* __restrict__ v_tail,
                                       const int* __restrict__ tail_slot, int num_decode) {
  constexpr int D = 128;
  constexpr int NL = (V_ROWS * (D / 8) + 255) / 256;  // row pieces per thread
  __shared__ bf16 tile[V_ROWS][D];
  __shared__ int64_t sl_s[V_ROWS + 1];  // slots[t0 - 1 + i] (-1 outside the batch)
  __shared__ int lead_n[V_SPAN];  // run length if the token leads a run, else 0
  __shared__ int lead_list[V_SPAN];
  __shared__ int n_leads;
  const int vh = span_id % Hkv;
  const int t0 = (span_id / Hkv) * V_SPAN;
  const int rows = min(V_ROWS, T - t0);
  const int tid = threadIdx.x;
  const bf16* src = qkv + (size_t)t0 * qkv_stride + (Hq + Hkv + vh) * D;
  bf16x8 rv[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int i = min(tid + 256 * j, rows * (D / 8) - 1);
    rv[j] = *reinterpret_cast<const bf16x8*>(src + (size_t)(i >> 4) * qkv_stride + (i & 15) * 8);
  }
  int64_t sv = -1;
  if (tid <= V_ROWS) {
    const int t = t0 - 1 + tid;
    if (t >= 0 && t < T) sv = slots[t];
  }
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int i = tid + 256 * j;
    if (i < rows * (D / 8)) *reinterpret_cast<bf16x8*>(&tile[i >> 4][(i & 15) * 8]) = rv[j];
  }
  if (tid <= V_ROWS) sl_s[tid] = sv;
  __syncthreads();
  if (tid < V_SPAN) {
    const int t = t0 + tid;
    int n = 0;
    if (t < T) {
      const int64_t s = sl_s[tid + 1];
      if (s >= 0 && (t == 0 || (s & 7) == 0 || sl_s[tid] != s - 1)) {
        n = 1;
        const int lim = 8 - (int)(s & 7);
        while (n < lim && t + n < T && sl_s[tid + 1 + n] == s + n) ++n;
      }
    }
    lead_n[tid] = n;
    // wave 0 holds the 64 span tokens: compact the leaders with a ballot
    const uint64_t m = __ballot(n > 0);
    if (n > 0) lead_list[__popcll(m & ((1ull << tid) - 1))] = tid;
    if (tid == 0) n_leads = __popcll(m);
  }
  __syncthreads();
  const int half = tid >> 7, d = tid & 127;
  for (int j = half; j < n_leads; j += 2) {
    const int i = lead_list[j];
    const int n = lead_n[i];
    const int t = t0 + i;
    const int64_t s = sl_s[i + 1];
    const int64_t blk = s / BS;
    const int off = (int)(s % BS);
    const int i0 = off & 7;
    const size_t g = ((size_t)blk * Hkv + vh) * D * BS + (off >> 3) * D * 8 + d * 8;
    // V tail (bf16): this sequence's partial group, token-major; element (token k, dim d)
    const int tsl = (!F8 && v_tail != nullptr) ? tail_slot[t] : -1;
    bf16* trow = tsl >= 0 ? v_tail + ((size_t)tsl * Hkv + vh) * 8 * D + d : nullptr;
    if (tsl >= 0 && t < num_decode && i0 + n == 8 && n < 8) {
      // a decode row completing its group: the group's earlier tokens live in the tail (decode
      // steps write no partial V lines) -> the whole [D][8] group, 16 full lines
      bf16x8 v;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = k < i0 ? trow[(size_t)k * D] : tile[i + k - i0][d];
      *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(v_cache) + g) = v;
      continue;
    }
    if (tsl >= 0 && i0 + n < 8) {
      // the group stays partial after this step: its tokens also go to the tail, where the
      // decode readers (and the step that completes the group) take them from
      for (int k = 0; k < n; ++k) trow[(size_t)(i0 + k) * D] = tile[i + k][d];
    }
    if (n == 8) {
      bf16x8 v;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = tile[i + k][d];
      if constexpr (F8) {
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        u32x2 w;
        w[0] = f32x4_to_fp8x4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
        w[1] = f32x4_to_fp8x4((float)v[4], (float)v[5], (float)v[6], (float)v[7]);
        *reinterpret_cast<u32x2*>(reinterpret_cast<uint8_t*>(v_cache) + g) = w;
      } else {
        *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(v_cache) + g) = v;
      }
    } else {
      for (int k = 0; k < n; ++k) {
        const size_t e = g + (off & 7) + k;
        if constexpr (F8)
          reinterpret_cast<uint8_t*>(v_cache)[e] = f32_to_fp8((float)tile[i + k][d]);
        else
          reinterpret_cast<bf16*>(v_cache)[e] = tile[i + k][d];
      }
    }
  }
}

// v role for decode batches (one new token per sequence: every run is a single token, so
// the span role's leader scan degenerates into one serial scatter per token): 16 lanes per
// (token, kv head), lane i writes dims [8i, 8i+8) of the token's slot.
template <bool F8>
__device__ __forceinline__ void v_item(const bf16* __restrict__ qkv, int qkv_stride,
                                       void* __restrict__ v_cache,
                                       const int64_t* __restrict__ slots, int T, int Hq, int Hkv,
                                       int BS, int vblk) {
  constexpr int D = 128;
  const int item = (vblk * 256 + threadIdx.x) >> 4;
  const int li = threadIdx.x & 15;
  if (item >= T * Hkv) return;
  const int t = item / Hkv, vh = item % Hkv;
  const int64_t slot = slots[t];
  if (slot < 0) return;
  const bf16x8 v = *reinterpret_cast<const bf16x8*>(qkv + (size_t)t * qkv_stride +
                                                    (Hq + Hkv + vh) * D + 8 * li);
  const int64_t blk = slot / BS;
  const int off = (int)(slot % BS);
  const size_t e = ((size_t)blk * Hkv + vh) * D * BS + (off >> 3) * D * 8 + (off & 7) +
                   (size_t)(8 * li) * 8;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if constexpr (F8) reinterpret_cast<uint8_t*>(v_cache)[e + 8 * k] = f32_to_fp8((float)v[k]);
    else reinterpret_cast<bf16*>(v_cache)[e + 8 * k] = v[k];
  }
}

template <bool F8>
__global__ __launch_bounds__(256) void qk_norm_rope_cache_kernel(
    const bf16* __restrict__ qkv, int qkv_stride, bf16* __restrict__ q_out,
    void* __restrict__ k_cache, void* __restrict__ v_cache, const int64_t* __restrict__ positions,
    const int64_t* __restrict__ slots, const float* __restrict__ cos_sin,
    const bf16* __restrict__ q_w, const bf16* __restrict__ k_w, int T, int Hq, int Hkv, int BS,
    float eps, int apply_rope, int qk_blocks, int v_per_token, bf16* __restrict__ v_tail,
    const int* __restrict__ tail_slot, int num_decode, int q_rows) {
  if ((int)blockIdx.x < qk_blocks)
    qk_tok<F8>(qkv, qkv_stride, q_out, k_cache, positions, slots, cos_sin, q_w, k_w, T, Hq, Hkv,
               BS, eps, apply_rope, q_rows);
  else if (v_per_token)
    v_item<F8>(qkv, qkv_stride, v_cache, slots, T, Hq, Hkv, BS, blockIdx.x - qk_blocks);
  else
    v_span<F8>(qkv, qkv_stride, v_cache, slots, T, Hq, Hkv, BS, blockIdx.x - qk_blocks, v_tail,
               tail_slot, num_decode);
}

void launch_qk_norm_rope_cache(const void* qkv, int qkv_stride, void* q_out, void* k_cache,
                               void* v_cache, const int64_t* positions, const int64_t* slots,
                               const float* cos_sin, const void* q_w, const void* k_w, int T,
                               int Hq, int Hkv, int D, int BS, float eps, int apply_rope,
                               hipStream_t s, int kv_fp8, int v_per_token, void* v_tail,
                               const int* tail_slot, int num_decode, int q_rows) {
  if (T == 0 || D != 128) return;
  if (v_per_token || kv_fp8) v_tail = nullptr;  // the tail is a bf16, span-role feature
  const int qk_blocks = (T + 15) / 16;  // 16 tokens per workgroup (qk_tok)
  const int v_blocks = v_per_token ? (int)(((long)T * Hkv * 16 + 255) / 256)
                                   : ((T + V_SPAN - 1) / V_SPAN) * Hkv;
  const dim3 grid(qk_blocks + v_blocks);
#define QKR(F8)                                                                                 \
  qk_norm_rope_cache_kernel<F8><<<grid, 256, 0, s>>>(                                           \
      (const bf16*)qkv, qkv_stride, (bf16*)q_out, k_cache, v_cache, positions, slots, cos_sin, \
      (const bf16*)q_w, (const bf16*)k_w, T, Hq, Hkv, BS, eps, apply_rope, qk_blocks, v_per_token, \
      (bf16*)v_tail, tail_slot, num_decode, q_rows)
  if (kv_fp8) QKR(true); else QKR(false);
#undef QKR
}

// Plain scatter of already-final K/V rows into the paged cache (used by the
// P/D KV receiver and by tests).  k, v: [T, Hkv, D].
template <int D, bool F8>
__global__ __launch_bounds__(256) void reshape_and_cache_kernel(
    const bf16* __restrict__ k, const bf16* __restrict__ v, void* __restrict__ k_cache,
    void* __restrict__ v_cache, const int64_t* __restrict__ slots, int T, int Hkv, int BS) {
  constexpr int LPH = D / 8;
  const int item = (blockIdx.x * 256 + threadIdx.x) / LPH;
  const int li = threadIdx.x % LPH;
  if (item >= T * Hkv) return;
  const int t = item / Hkv, h = item % Hkv;
  const int64_t slot = slots[t];
  if (slot < 0) return;
  const int64_t blk = slot / BS;
  const int off = (int)(slot % BS);
  bf16x8 kv = *reinterpret_cast<const bf16x8*>(k + ((size_t)t * Hkv + h) * D + 8 * li);
  bf16x8 vv = *reinterpret_cast<const bf16x8*>(v + ((size_t)t * Hkv + h) * D + 8 * li);
  const size_t ke = ((size_t)blk * Hkv + h) * BS * D + k_swz_offset(off) + k_dim_offset(8 * li);
  const size_t ve = ((size_t)blk * Hkv + h) * D * BS + (off >> 3) * D * 8 + (off & 7);
  if constexpr (F8) {
    uint32_t* kd = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(k_cache) + ke);
    kd[0] = f32x4_to_fp8x4((float)kv[0], (float)kv[1], (float)kv[2], (float)kv[3]);
    kd[1] = f32x4_to_fp8x4((float)kv[4], (float)kv[5], (float)kv[6], (float)kv[7]);
    uint8_t* vd = reinterpret_cast<uint8_t*>(v_cache) + ve;
#pragma unroll
    for (int j = 0; j < 8; ++j) vd[(size_t)(8 * li + j) * 8] = f32_to_fp8((float)vv[j]);
  } else {
    *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(k_cache) + ke) = kv;
    bf16* vd = reinterpret_cast<bf16*>(v_cache) + ve;
#pragma unroll
    for (int j = 0; j < 8; ++j) vd[(size_t)(8 * li + j) * 8] = vv[j];
  }
}

void launch_reshape_and_cache(const void* k, const void* v, void* k_cache, void* v_cache,
                              const int64_t* slots, int T, int Hkv, int D, int BS, hipStream_t s,
                              int kv_fp8) {
  if (T == 0 || D != 128) return;
  const long threads = (long)T * Hkv * (D / 8);
  dim3 grid((threads + 255) / 256);
  if (kv_fp8)
    reshape_and_cache_kernel<128, true><<<grid, 256, 0, s>>>((const bf16*)k, (const bf16*)v,
                                                            k_cache, v_cache, slots, T, Hkv, BS);
  else
    reshape_and_cache_kernel<128, false><<<grid, 256, 0, s>>>((const bf16*)k, (const bf16*)v,
                                                             k_cache, v_cache, slots, T, Hkv, BS);
}

}  // namespace akap
