// QKV projection GEMM with the per-head epilogue of a decode attention layer, for gfx950:
//   y = X[M,K] . W[N,K]^T (rows optionally scaled by the input RMSNorm's rsqrt(ss_in/K+eps)),
//   then per head: q/k RMSNorm (Qwen3 q_norm / k_norm, optional), NeoX RoPE, and
//   q -> q_out [M, Hq, 128];  k, v -> the new token's slot of the paged K / V caches.
//
// Why: the decode attention kernel used to do this itself (paged_attn_decode_kernel FUSED),
// but there the prologue is a chain of dependent loads (seq_lens -> positions -> cos/sin,
// the qkv row, the cache write, a barrier) at the START of every (sequence, kv head)
// workgroup -- 2048 workgroups in two rounds at B = 256, so ~2 x 4 us of the HBM-bound
// K/V stream is spent waiting: 114.1 us vs 105.8 us for the same attention on a ready q
// (profiles/r2_attn_fused_ab.log).  In the GEMM the same work is a short epilogue on
// values already in registers, and the attention kernel starts streaming immediately.
//
// Geometry: one workgroup = BM rows x ONE head (128 columns), 4 waves each owning 32
// columns (2 x BM/16 MFMA 16x16x32 tiles), BK = 64, operands staged by global_load_lds into
// an NS-slot LDS ring (counted vmcnt + raw s_barrier per k-step, XOR swizzle on the DMA
// source address and on the fragment reads -- the gdgemm.hip structure).  Epilogue: the
// bf16-rounded tile goes through LDS; 8 threads per row x 16 dims each do the norm's row
// sum (xor-shuffles over the 8) and the RoPE pair exchange (dims d, d+64 sit in threads j,
// j^4), then 16-byte q / K stores and the V cache's 8-token-group scatter.
#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int QBK = 64;
constexpr int QD = 128;
constexpr int QEP = QD + 4;  // epilogue LDS row pitch (floats)

__device__ __forceinline__ int qswz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }

__device__ __forceinline__ void qglds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0,
                                   0);
}

template <int N_>
__device__ __forceinline__ void qwait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

template <int BM, int NS, bool F8>
__global__ __launch_bounds__(256, 1) void qkv_rope_gemm_kernel(QkvRopeArgs p) {
  constexpr int MI = BM / 16;            // 16-row MFMA tiles per wave
  constexpr int GA = BM / 32, GW = 4;    // DMA instructions per wave per k-step
  constexpr int G = GA + GW;
  constexpr int SU = (BM + QD) * 8;      // ring slot, 16-B units
  constexpr int LDS_UNITS = NS * SU > BM * QEP / 4 ? NS * SU : BM * QEP / 4;
  __shared__ bf16x8 lds[LDS_UNITS];

  const int H = p.Hq + 2 * p.Hkv;
  const int tiles_m = (p.M + BM - 1) / BM;
  const int lt = xcd_remap(blockIdx.x, H * tiles_m);
  const int head = lt / tiles_m, tm = lt % tiles_m;  // a head's row tiles share an XCD
  const int m0 = tm * BM, n0 = head * QD;
  const int nk = p.K / QBK;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const bf16* X = static_cast<const bf16*>(p.X);
  const bf16* W = static_cast<const bf16*>(p.W);

  const int lr = lane >> 3, lc = (lane & 7) ^ (lane >> 3);
  const bf16* asrc[GA];
  const bf16* wsrc[GW];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int row = m0 + (w * GA + i) * 8 + lr;
    asrc[i] = X + (size_t)(row < p.M ? row : 0) * p.ldx + lc * 8;
  }
#pragma unroll
  for (int i = 0; i < GW; ++i) wsrc[i] = W + (size_t)(n0 + (w * GW + i) * 8 + lr) * p.ldw + lc * 8;
  auto issue = [&](int step) {
    bf16x8* slot = lds + (step % NS) * SU;
    const int k0 = step * QBK;
#pragma unroll
    for (int i = 0; i < GA; ++i) qglds16(asrc[i] + k0, slot + (w * GA + i) * 64);
#pragma unroll
    for (int i = 0; i < GW; ++i) qglds16(wsrc[i] + k0, slot + BM * 8 + (w * GW + i) * 64);
  };

  // epilogue operand loaded ahead of the loop (hidden under it)
  float rs[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + i * 16 + fg * 4 + r;
      rs[i][r] = p.ss_in != nullptr ? p.ss_in[row < p.M ? row : 0] : 0.f;
    }

  f32x4 acc[MI][2];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s);
  for (int t = 0; t < nk; ++t) {
    if (t + NS - 2 < nk) qwait_vm<G * (NS - 2)>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // step t landed for every wave; slot t-1 is free
    if (t + NS - 1 < nk) issue(t + NS - 1);
    const bf16x8* slot = lds + (t % NS) * SU;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MI], bfr[2];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = slot[qswz(i * 16 + fr, ks * 4 + fg)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = slot[BM * 8 + qswz(w * 32 + j * 16 + fr, ks * 4 + fg)];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  // ---- epilogue: y = bf16(acc * row scale) -> LDS [BM][QEP] floats ----
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // ring no longer read by any wave
  float* E = reinterpret_cast<float*>(lds);
  const float inv_k = 1.f / (float)p.K;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float sc = p.ss_in != nullptr ? rsqrtf(rs[i][r] * inv_k + p.eps) : 1.f;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        E[(i * 16 + fg * 4 + r) * QEP + w * 32 + j * 16 + fr] = bf2f(f2bf(acc[i][j][r] * sc));
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  const int kind = head < p.Hq ? 0 : (head < p.Hq + p.Hkv ? 1 : 2);  // q | k | v
  const int kvh = kind == 1 ? head - p.Hq : head - p.Hq - p.Hkv;
  const bf16* nw = kind == 0 ? static_cast<const bf16*>(p.q_w)
                             : (kind == 1 ? static_cast<const bf16*>(p.k_w) : nullptr);
  const int j = tid & 7;  // dims 16j .. 16j+15 of the row
#pragma unroll
  for (int rb = 0; rb < BM; rb += 32) {
    const int lrow = rb + (tid >> 3);
    const int row = m0 + lrow;
    float x[16];
#pragma unroll
    for (int q = 0; q < 16; q += 4) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(&E[lrow * QEP + 16 * j + q]);
      x[q] = v[0]; x[q + 1] = v[1]; x[q + 2] = v[2]; x[q + 3] = v[3];
    }
    if (kind != 2) {
      if (nw != nullptr) {  // per-head RMSNorm (bf16-rounded, like the standalone kernel)
        float ss = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) ss += x[q] * x[q];
        ss += __shfl_xor(ss, 1, 8);
        ss += __shfl_xor(ss, 2, 8);
        ss += __shfl_xor(ss, 4, 8);
        const float inv = rsqrtf(ss / (float)QD + p.eps);
        const bf16x8 w0 = *reinterpret_cast<const bf16x8*>(nw + 16 * j);
        const bf16x8 w1 = *reinterpret_cast<const bf16x8*>(nw + 16 * j + 8);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          x[q] = bf2f(f2bf(x[q] * inv * bf2f(w0[q])));
          x[8 + q] = bf2f(f2bf(x[8 + q] * inv * bf2f(w1[q])));
        }
      }
      if (p.rope) {  // NeoX: (d, d+64) pairs live in threads j and j^4
        const int64_t pos = p.positions[row < p.M ? row : 0];
        const float* cs = p.cos_sin + (size_t)pos * QD + 16 * (j & 3);
        float c[16], s[16];
#pragma unroll
        for (int q = 0; q < 16; q += 4) {
          const f32x4 cv = *reinterpret_cast<const f32x4*>(cs + q);
          const f32x4 sv = *reinterpret_cast<const f32x4*>(cs + 64 + q);
          c[q] = cv[0]; c[q + 1] = cv[1]; c[q + 2] = cv[2]; c[q + 3] = cv[3];
          s[q] = sv[0]; s[q + 1] = sv[1]; s[q + 2] = sv[2]; s[q + 3] = sv[3];
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const float other = __shfl_xor(x[q], 4, 8);
          x[q] = j < 4 ? x[q] * c[q] - other * s[q] : x[q] * c[q] + other * s[q];
        }
      }
    }
    if (row >= p.M) continue;
    bf16x8 o0, o1;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      o0[q] = f2bf(x[q]);
      o1[q] = f2bf(x[8 + q]);
    }
    if (kind == 0) {
      bf16* qo = static_cast<bf16*>(p.q_out) + ((size_t)row * p.Hq + head) * QD + 16 * j;
      *reinterpret_cast<bf16x8*>(qo) = o0;
      *reinterpret_cast<bf16x8*>(qo + 8) = o1;
      continue;
    }
    const int64_t slot = p.slots[row];
    if (slot < 0) continue;
    const int64_t blk = slot / p.BS;
    const int off = (int)(slot % p.BS);
    if (kind == 1) {
      const size_t e = ((size_t)blk * p.Hkv + kvh) * p.BS * QD + k_swz_offset(off);
      const size_t e0 = e + k_dim_offset(16 * j), e1 = e + k_dim_offset(16 * j + 8);
      if constexpr (F8) {
        uint32_t* d0 = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(p.k_cache) + e0);
        uint32_t* d1 = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(p.k_cache) + e1);
        d0[0] = f32x4_to_fp8x4(x[0], x[1], x[2], x[3]);
        d0[1] = f32x4_to_fp8x4(x[4], x[5], x[6], x[7]);
        d1[0] = f32x4_to_fp8x4(x[8], x[9], x[10], x[11]);
        d1[1] = f32x4_to_fp8x4(x[12], x[13], x[14], x[15]);
      } else {
        *reinterpret_cast<bf16x8*>(static_cast<bf16*>(p.k_cache) + e0) = o0;
        *reinterpret_cast<bf16x8*>(static_cast<bf16*>(p.k_cache) + e1) = o1;
      }
    } else {
      const size_t e = ((size_t)blk * p.Hkv + kvh) * QD * p.BS + (off >> 3) * QD * 8 + (off & 7);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const size_t a = e + (size_t)(16 * j + q) * 8;
        if constexpr (F8) static_cast<uint8_t*>(p.v_cache)[a] = f32_to_fp8(x[q]);
        else static_cast<bf16*>(p.v_cache)[a] = f2bf(x[q]);
      }
    }
  }
}

bool qkv_rope_gemm_supported(int M, int K, int bm, int ns) {
  return M > 0 && K >= QBK && K % QBK == 0 && (bm == 32 || bm == 64) && (ns == 3 || ns == 6);
}

template <int BM, int NS>
static void qkv_launch(const QkvRopeArgs& p, int grid, hipStream_t st) {
  if (p.kv_fp8) qkv_rope_gemm_kernel<BM, NS, true><<<grid, 256, 0, st>>>(p);
  else qkv_rope_gemm_kernel<BM, NS, false><<<grid, 256, 0, st>>>(p);
}

void launch_qkv_rope_gemm(const QkvRopeArgs& p, int bm, int ns, hipStream_t st) {
  if (p.M == 0) return;
  const int grid = (p.Hq + 2 * p.Hkv) * ((p.M + bm - 1) / bm);
  if (bm == 64) {
    if (ns == 6) qkv_launch<64, 6>(p, grid, st);
    else qkv_launch<64, 3>(p, grid, st);
  } else {
    if (ns == 6) qkv_launch<32, 6>(p, grid, st);
    else qkv_launch<32, 3>(p, grid, st);
  }
}

}  // namespace akap
