// Fused post-QKV-projection epilogue for gfx950:
//   per-head RMSNorm on q and k (Qwen3; optional)  ->  NeoX rotary on q and k
//   -> q written contiguous [T, Hq, D]; k, v scattered into the paged KV cache.
//
// One pass over the QKV activations instead of three (norm, rope, cache write).
// D/8 lanes own one head: lane i holds dims [4i, 4i+4) and their rotary partners
// [D/2 + 4i, D/2 + 4i + 4) so the rotate-half pairing is lane-local.  cos/sin come
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

// True when batch token t belongs to an 8-token V slot group whose 8 tokens are all in the
// batch, consecutive (slots s0..s0+7, s0 % 8 == 0).  Written slots are never shared between
// sequences (shared prefix blocks are full and read-only), so consecutive slots imply one
// sequence's consecutive positions.
__device__ __forceinline__ bool v_group_complete(const int64_t* __restrict__ slots, int t, int T,
                                                 int64_t slot) {
  const int r = (int)(slot & 7);
  const int g0 = t - r;
  if (g0 < 0 || g0 + 7 >= T) return false;
  return slots[g0] == slot - r && slots[g0 + 7] == slot - r + 7;
}

template <int D, bool F8>
__global__ __launch_bounds__(256) void qk_norm_rope_cache_kernel(
    const bf16* __restrict__ qkv, int qkv_stride, bf16* __restrict__ q_out,
    void* __restrict__ k_cache, void* __restrict__ v_cache, const int64_t* __restrict__ positions,
    const int64_t* __restrict__ slots, const float* __restrict__ cos_sin,
    const bf16* __restrict__ q_w, const bf16* __restrict__ k_w, int T, int Hq, int Hkv, int BS,
    float eps, int apply_rope) {
  constexpr int LPH = D / 8;  // lanes per head
  constexpr int HALF = D / 2;
  const int heads_total = Hq + 2 * Hkv;
  const int item = (blockIdx.x * 256 + threadIdx.x) / LPH;
  const int li = threadIdx.x % LPH;
  if (item >= T * heads_total) return;
  const int t = item / heads_total;
  const int h = item % heads_total;
  const bf16* src = qkv + (size_t)t * qkv_stride + h * D;
  bf16x4 a = *reinterpret_cast<const bf16x4*>(src + 4 * li);
  bf16x4 b = *reinterpret_cast<const bf16x4*>(src + HALF + 4 * li);
  float xa[4], xb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) { xa[j] = bf2f(a[j]); xb[j] = bf2f(b[j]); }

  const bool is_q = h < Hq;
  const bool is_k = !is_q && h < Hq + Hkv;
  if (is_q || is_k) {
    const bf16* nw = is_q ? q_w : k_w;
    if (nw != nullptr) {
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) ss += xa[j] * xa[j] + xb[j] * xb[j];
#pragma unroll
      for (int o = LPH / 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, LPH);
      const float inv = rsqrtf(ss / (float)D + eps);
      bf16x4 wa = *reinterpret_cast<const bf16x4*>(nw + 4 * li);
      bf16x4 wb = *reinterpret_cast<const bf16x4*>(nw + HALF + 4 * li);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // round-trip through bf16 like the reference module (norm output is bf16)
        xa[j] = bf2f(f2bf(xa[j] * inv * bf2f(wa[j])));
        xb[j] = bf2f(f2bf(xb[j] * inv * bf2f(wb[j])));
      }
    }
    if (apply_rope) {
      const float* cs = cos_sin + (size_t)positions[t] * D;
      f32x4 c = *reinterpret_cast<const f32x4*>(cs + 4 * li);
      f32x4 s = *reinterpret_cast<const f32x4*>(cs + HALF + 4 * li);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x1 = xa[j], x2 = xb[j];
        xa[j] = x1 * c[j] - x2 * s[j];
        xb[j] = x2 * c[j] + x1 * s[j];
      }
    }
  }
  bf16x4 oa, ob;
#pragma unroll
  for (int j = 0; j < 4; ++j) { oa[j] = f2bf(xa[j]); ob[j] = f2bf(xb[j]); }
  if (is_q) {
    bf16* dst = q_out + ((size_t)t * Hq + h) * D;
    *reinterpret_cast<bf16x4*>(dst + 4 * li) = oa;
    *reinterpret_cast<bf16x4*>(dst + HALF + 4 * li) = ob;
    return;
  }
  const int64_t slot = slots[t];
  if (slot < 0) return;
  const int64_t blk = slot / BS;
  const int off = (int)(slot % BS);
  if (is_k) {
    const int kh = h - Hq;
    const size_t e = ((size_t)blk * Hkv + kh) * BS * D + k_swz_offset(off);
    if constexpr (F8) {
      uint8_t* dst = reinterpret_cast<uint8_t*>(k_cache) + e;
      // from the bf16-rounded values (same rounding chain as the bf16 cache + reference)
      *reinterpret_cast<uint32_t*>(dst + k_dim_offset(4 * li)) =
          f32x4_to_fp8x4((float)oa[0], (float)oa[1], (float)oa[2], (float)oa[3]);
      *reinterpret_cast<uint32_t*>(dst + k_dim_offset(HALF + 4 * li)) =
          f32x4_to_fp8x4((float)ob[0], (float)ob[1], (float)ob[2], (float)ob[3]);
    } else {
      bf16* dst = reinterpret_cast<bf16*>(k_cache) + e;
      *reinterpret_cast<bf16x4*>(dst + k_dim_offset(4 * li)) = oa;
      *reinterpret_cast<bf16x4*>(dst + k_dim_offset(HALF + 4 * li)) = ob;
    }
  } else {
    // tokens of a complete 8-token slot group are written by v_group_write_kernel as
    // 16-byte vectors; only stragglers (chunk edges, decode tokens) scatter 2-byte stores
    if (v_group_complete(slots, t, T, slot)) return;
    const int vh = h - Hq - Hkv;
    const size_t e = ((size_t)blk * Hkv + vh) * D * BS + (off >> 3) * D * 8 + (off & 7);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (F8) {
        uint8_t* dst = reinterpret_cast<uint8_t*>(v_cache) + e;
        dst[(size_t)(4 * li + j) * 8] = f32_to_fp8((float)oa[j]);
        dst[(size_t)(HALF + 4 * li + j) * 8] = f32_to_fp8((float)ob[j]);
      } else {
        bf16* dst = reinterpret_cast<bf16*>(v_cache) + e;
        dst[(size_t)(4 * li + j) * 8] = oa[j];
        dst[(size_t)(HALF + 4 * li + j) * 8] = ob[j];
      }
    }
  }
}

// V cache groups are [D][8 tokens]: a token alone can only be written as D scattered
// 2-byte stores.  When the batch holds all 8 tokens of a slot group (prefill chunks), a
// thread per dim gathers the 8 values (each read coalesced across the wave) and writes one
// 16-byte vector.  grid = (ceil(T / 64), Hkv), 128 threads = one per dim.
template <bool F8>
__global__ __launch_bounds__(128) void v_group_write_kernel(const bf16* __restrict__ qkv,
                                                            int qkv_stride,
                                                            void* __restrict__ v_cache,
                                                            const int64_t* __restrict__ slots,
                                                            int T, int Hq, int Hkv, int BS) {
  constexpr int D = 128;
  const int vh = blockIdx.y;
  const int d = threadIdx.x;
  const int t_end = min(T, (int)(blockIdx.x + 1) * 64);
  for (int t = blockIdx.x * 64; t < t_end; ++t) {
    const int64_t slot = slots[t];
    if (slot < 0 || (slot & 7) != 0 || !v_group_complete(slots, t, T, slot)) continue;
    const bf16* src = qkv + (size_t)t * qkv_stride + (Hq + Hkv + vh) * D + d;
    bf16x8 g8;
#pragma unroll
    for (int i = 0; i < 8; ++i) g8[i] = src[(size_t)i * qkv_stride];
    const int64_t blk = slot / BS;
    const int off = (int)(slot % BS);
    const size_t e = ((size_t)blk * Hkv + vh) * D * BS + (off >> 3) * D * 8 + d * 8;
    if constexpr (F8) {
      uint32_t* dst = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(v_cache) + e);
      dst[0] = f32x4_to_fp8x4((float)g8[0], (float)g8[1], (float)g8[2], (float)g8[3]);
      dst[1] = f32x4_to_fp8x4((float)g8[4], (float)g8[5], (float)g8[6], (float)g8[7]);
    } else {
      *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(v_cache) + e) = g8;
    }
  }
}

void launch_qk_norm_rope_cache(const void* qkv, int qkv_stride, void* q_out, void* k_cache,
                               void* v_cache, const int64_t* positions, const int64_t* slots,
                               const float* cos_sin, const void* q_w, const void* k_w, int T,
                               int Hq, int Hkv, int D, int BS, float eps, int apply_rope,
                               hipStream_t s, int kv_fp8) {
  if (T == 0 || D != 128) return;
  const long items = (long)T * (Hq + 2 * Hkv);
  const long threads = items * (D / 8);
  dim3 grid((threads + 255) / 256);
#define QKR(F8)                                                                                 \
  qk_norm_rope_cache_kernel<128, F8><<<grid, 256, 0, s>>>(                                      \
      (const bf16*)qkv, qkv_stride, (bf16*)q_out, k_cache, v_cache, positions, slots, cos_sin, \
      (const bf16*)q_w, (const bf16*)k_w, T, Hq, Hkv, BS, eps, apply_rope)
  if (kv_fp8) QKR(true); else QKR(false);
#undef QKR
  if (T >= 8) {
    const dim3 g2((T + 63) / 64, Hkv);
    if (kv_fp8)
      v_group_write_kernel<true><<<g2, 128, 0, s>>>((const bf16*)qkv, qkv_stride, v_cache, slots,
                                                     T, Hq, Hkv, BS);
    else
      v_group_write_kernel<false><<<g2, 128, 0, s>>>((const bf16*)qkv, qkv_stride, v_cache,
                                                      slots, T, Hq, Hkv, BS);
  }
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
