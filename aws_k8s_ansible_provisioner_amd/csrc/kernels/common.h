// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernels.
//
// Everything here assumes wave64, 16-byte vector memory ops and bf16 storage.
// No CUDA compatibility layer: these are CDNA4 intrinsics used directly.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace akap {

constexpr int kWave = 64;

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

template <typename T>
__device__ __forceinline__ T ld_nt(const T* p) {
  return __builtin_nontemporal_load(p);
}

// Full-wave reductions (64 lanes) using DPP/permute via __shfl_xor.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Wave-uniform reductions on DPP (VALU lane swaps, no LDS round trip): xor 1 and 2 as quad
// permutes, 4 and 8 as the half-row / row mirrors (each leaves the 4- then 8- then 16-lane
// groups uniform), then the four 16-lane rows through v_readlane.  For per-tile reductions in
// streaming loops, where __shfl_xor's ds_bpermute chain (6 dependent LDS round trips) stalls.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));   // quad_perm [1,0,3,2]
  v = fmaxf(v, dpp_mov<0x4E>(v));   // quad_perm [2,3,0,1]
  v = fmaxf(v, dpp_mov<0x141>(v));  // row_half_mirror
  v = fmaxf(v, dpp_mov<0x140>(v));  // row_mirror
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x141>(v);
  v += dpp_mov<0x140>(v);
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}

// Block-wide sum for blockDim.x a multiple of 64, <= 1024. `scratch` needs 16 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  v = wave_sum(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = lane < nw ? scratch[lane] : 0.f;
  r = wave_sum(r);
  __syncthreads();
  return r;
}

__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  v = wave_max(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = lane < nw ? scratch[lane] : -INFINITY;
  r = wave_max(r);
  __syncthreads();
  return r;
}

// XCD-aware bijective remap of a 1-D workgroup id (cdna_hip_programming §5, T1):
// consecutive logical tiles land on the same XCD (shared L2).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

// Counter-based RNG (splitmix-style hash), deterministic per (seed, a, b).
__device__ __forceinline__ uint32_t hash3(uint64_t seed, uint32_t a, uint32_t b) {
  uint64_t x = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(a + 1)) ^ ((uint64_t)b << 32 | b);
  x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27; x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)(x >> 32);
}

__device__ __forceinline__ float uniform01(uint64_t seed, uint32_t a, uint32_t b) {
  // strictly inside (0, 1): -log(u) and -log(-log(u)) stay finite (u = 1 would make a Gumbel
  // draw +inf, i.e. a uniformly random token once in 2^24 elements)
  return ((float)(hash3(seed, a, b) >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

// ---- paged K cache layout (D = 128) --------------------------------------------------
// Within one (block, kv head) of BS tokens (BS % 32 == 0), each 32-token chunk is stored as
// [tile tt (2)][k-step cc (4)][row r (16)][32 dims]: the exact operand order of the
// attention kernels' S^T = K.Q^T MFMA tiles, whose row r of tile tt is chunk token
// 8*(r>>2) + 4*tt + (r&3).  Element offset of (token `off`, dim 0) within the block-head;
// dim d lives at + (d/32)*512 + d%32.
__host__ __device__ __forceinline__ int k_swz_offset(int off) {
  const int o = off & 31;
  const int tt = (o >> 2) & 1;
  const int r = ((o >> 3) << 2) | (o & 3);
  return (off >> 5) * 32 * 128 + tt * 16 * 128 + r * 32;
}
__host__ __device__ __forceinline__ int k_dim_offset(int d) { return (d >> 5) * 512 + (d & 31); }

// ---- FP8 (OCP e4m3fn) KV-cache storage ---------------------------------------------------
// Optional 1-byte KV cache (--kv-cache-dtype fp8, per-tensor scale 1.0): halves the bytes
// the HBM-bound decode attention streams.  Values are clamped to +-448 (e4m3fn max) and
// rounded to nearest even on store; loads widen 8 bytes to 8 bf16 (exact: every e4m3 value
// is representable in bf16) right before the bf16 MFMAs.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ bf16x8 fp8x8_to_bf16x8(uint32_t lo, uint32_t hi) {
  const bf16x2_t a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, 1.0f, false);
  const bf16x2_t b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, 1.0f, true);
  const bf16x2_t c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, 1.0f, false);
  const bf16x2_t d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, 1.0f, true);
  return bf16x8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}

__device__ __forceinline__ float fp8_clamp(float x) { return fminf(fmaxf(x, -448.f), 448.f); }

// 4 floats -> 4 fp8 bytes (little-endian element order) in one 32-bit word
__device__ __forceinline__ uint32_t f32x4_to_fp8x4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(fp8_clamp(a), fp8_clamp(b), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(fp8_clamp(c), fp8_clamp(d), w, true);
  return (uint32_t)w;
}

__device__ __forceinline__ uint8_t f32_to_fp8(float a) {
  return (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(fp8_clamp(a), 0.f, 0, false) & 0xff);
}

// 8 consecutive cache elements starting at element `off` -> bf16x8
template <bool F8, bool NT>
__device__ __forceinline__ bf16x8 ld_kv8(const void* base, size_t off) {
  if constexpr (F8) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const u32x2* p = reinterpret_cast<const u32x2*>(reinterpret_cast<const uint8_t*>(base) + off);
    u32x2 v;
    if constexpr (NT) v = __builtin_nontemporal_load(p);
    else v = *p;
    return fp8x8_to_bf16x8(v[0], v[1]);
  } else {
    const bf16x8* p = reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(base) + off);
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
  }
}

}  // namespace akap
