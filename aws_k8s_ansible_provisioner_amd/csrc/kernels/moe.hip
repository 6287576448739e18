// Mixture-of-experts routing kernels for gfx950.
//  * moe_topk_softmax: router logits [T, E] -> softmax -> top-k (+ optional renorm).
//    One lane per token for E <= 32 (Mixtral), one wave per token above (Qwen3-MoE, E <= 256).
//  * moe_align: groups the T*K (token, expert) pairs by expert, padding every
//    expert's segment to a multiple of the grouped-GEMM row tile so each tile of
//    the sorted list belongs to exactly one expert.  Single workgroup, LDS counts.
#include "common.h"
#include "kernels.h"

namespace akap {

// softmax over E logits (read through x(e)) -> top-K (ties -> lowest expert id), optional
// renormalisation of the K weights
template <typename F>
__device__ __forceinline__ void topk_softmax_row(F x, int E, int K, float* __restrict__ w_out,
                                                 int32_t* __restrict__ id_out, int renorm) {
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) mx = fmaxf(mx, x(e));
  float z = 0.f;
  for (int e = 0; e < E; ++e) z += __expf(x(e) - mx);
  const float invz = 1.f / z;
  float wsum = 0.f;
  // selection by repeated scan (K is tiny: 1..8)
  uint64_t taken_lo = 0, taken_hi = 0, taken_2 = 0, taken_3 = 0;
  for (int k = 0; k < K; ++k) {
    float best = -INFINITY;
    int bi = 0;
    for (int e = 0; e < E; ++e) {
      const uint64_t bit = 1ull << (e & 63);
      const uint64_t word = e < 64 ? taken_lo : e < 128 ? taken_hi : e < 192 ? taken_2 : taken_3;
      if (word & bit) continue;
      const float v = x(e);
      if (v > best) { best = v; bi = e; }
    }
    const uint64_t bit = 1ull << (bi & 63);
    if (bi < 64) taken_lo |= bit; else if (bi < 128) taken_hi |= bit;
    else if (bi < 192) taken_2 |= bit; else taken_3 |= bit;
    const float w = __expf(best - mx) * invz;
    w_out[k] = w;
    id_out[k] = bi;
    wsum += w;
  }
  if (renorm) {
    const float inv = 1.f / wsum;
    for (int k = 0; k < K; ++k) w_out[k] *= inv;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void moe_topk_softmax_kernel(const T* __restrict__ logits,
                                                               int ld, int E, int K,
                                                               float* __restrict__ topk_w,
                                                               int32_t* __restrict__ topk_ids,
                                                               int Tn, int renorm) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= Tn) return;
  const T* x = logits + (size_t)t * ld;
  topk_softmax_row([&](int e) { return (float)x[e]; }, E, K, topk_w + (size_t)t * K,
                   topk_ids + (size_t)t * K, renorm);
}

// Router GEMM + softmax + top-k in one launch for E <= kRouterMaxE experts: one workgroup per
// token.  Its 256 threads take 8-element slices of the hidden row and of every router row
// (the E x d router, 64 KB for Mixtral, stays L2-resident), the E dot products are reduced
// across the workgroup, and the logits are rounded to bf16 like the separate F.linear's
// output before the softmax.  Replaces a hipBLASLt launch (M x 8 output: 13.5 us at M = 128)
// plus the top-k launch (profiles/r2_mixtral_bench_kernel_stats.md).
constexpr int kRouterMaxE = 16;

__global__ __launch_bounds__(256) void moe_router_topk_kernel(const bf16* __restrict__ h, int ldh,
                                                              const bf16* __restrict__ W, int d,
                                                              int E, int K,
                                                              float* __restrict__ topk_w,
                                                              int32_t* __restrict__ topk_ids,
                                                              int renorm) {
  __shared__ float part[4][kRouterMaxE];
  __shared__ float logit[kRouterMaxE];
  const int t = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bf16* x = h + (size_t)t * ldh;
  float acc[kRouterMaxE];
#pragma unroll
  for (int e = 0; e < kRouterMaxE; ++e) acc[e] = 0.f;
  for (int c = tid; c < d / 8; c += 256) {
    const bf16x8 xv = *reinterpret_cast<const bf16x8*>(x + 8 * c);
#pragma unroll
    for (int e = 0; e < kRouterMaxE; ++e) {
      if (e < E) {
        const bf16x8 wv = *reinterpret_cast<const bf16x8*>(W + (size_t)e * d + 8 * c);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[e] += bf2f(xv[i]) * bf2f(wv[i]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < kRouterMaxE; ++e) {
    if (e < E) {
      float v = acc[e];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0) part[w][e] = v;
    }
  }
  __syncthreads();
  if (tid < E) logit[tid] = bf2f(f2bf(part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid]));
  __syncthreads();
  if (tid == 0)
    topk_softmax_row([&](int e) { return logit[e]; }, E, K, topk_w + (size_t)t * K,
                     topk_ids + (size_t)t * K, renorm);
}

bool moe_router_topk_supported(int E, int d) { return E >= 1 && E <= kRouterMaxE && d % 8 == 0; }

void launch_moe_router_topk(const void* h, int ldh, const void* W, int d, int E, int K,
                            float* topk_w, int32_t* topk_ids, int T, int renormalize,
                            hipStream_t s) {
  if (T == 0) return;
  moe_router_topk_kernel<<<T, 256, 0, s>>>((const bf16*)h, ldh, (const bf16*)W, d, E, K, topk_w,
                                           topk_ids, renormalize);
}

// Many-expert routing (Qwen3-MoE: E = 128, K = 8): one WAVE per token.  Lane l holds logits
// l, l + 64, l + 128, l + 192 (E <= 256); max and sum-of-exp are wave reductions; each of the
// K picks is a wave argmax over the lanes' best unpicked logit (ties -> lowest expert id, as in
// topk_softmax_row).  The one-lane-per-token kernel above spends E x K serial steps per lane:
// 189 us per call at T = 256, E = 128, K = 8 (profiles/r4_qwen3_moe_kernel_stats.md).
__device__ __forceinline__ void wave_argmax(float& v, int& idx) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (ov > v || (ov == v && oi < idx)) {
      v = ov;
      idx = oi;
    }
  }
}

__global__ __launch_bounds__(256) void moe_topk_softmax_wave_kernel(
    const bf16* __restrict__ logits, int ld, int E, int K, float* __restrict__ topk_w,
    int32_t* __restrict__ topk_ids, int Tn, int renorm) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= Tn) return;  // wave-uniform
  const bf16* x = logits + (size_t)t * ld;
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = lane + 64 * j;
    v[j] = e < E ? bf2f(x[e]) : -INFINITY;
  }
  float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float z = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) z += lane + 64 * j < E ? __expf(v[j] - mx) : 0.f;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) z += __shfl_xor(z, o, 64);
  const float invz = 1.f / z;
  float my_w = 0.f, wsum = 0.f;
  int my_id = 0;
  for (int k = 0; k < K; ++k) {
    float best = v[0];
    int bi = lane;
#pragma unroll
    for (int j = 1; j < 4; ++j)
      if (v[j] > best) {  // strict: the lower expert id of a lane wins ties
        best = v[j];
        bi = lane + 64 * j;
      }
    wave_argmax(best, bi);
    if ((bi & 63) == lane) v[bi >> 6] = -INFINITY;  // the owning lane retires the pick
    const float w = __expf(best - mx) * invz;
    wsum += w;
    if (lane == k) {
      my_w = w;
      my_id = bi;
    }
  }
  if (lane < K) {
    topk_w[(size_t)t * K + lane] = renorm ? my_w / wsum : my_w;
    topk_ids[(size_t)t * K + lane] = my_id;
  }
}

void launch_moe_topk_softmax(const void* logits, int ld, int E, int K, float* topk_w,
                             int32_t* topk_ids, int T, int renormalize, hipStream_t s) {
  if (T == 0) return;
  if (E > 32) {
    moe_topk_softmax_wave_kernel<<<(T + 3) / 4, 256, 0, s>>>(
        (const bf16*)logits, ld, E, K, topk_w, topk_ids, T, renormalize);
    return;
  }
  moe_topk_softmax_kernel<bf16><<<(T + 255) / 256, 256, 0, s>>>(
      (const bf16*)logits, ld, E, K, topk_w, topk_ids, T, renormalize);
}

// sorted_ids: [n + E*(block-1)] rounded, filled with n (sentinel) for padding.
// inv[i] = position of flat (token, k) index i in the sorted list (for the combine);
// tile_expert[t] = expert of row tile t (block rows each), -1 past the last tile.
__global__ __launch_bounds__(1024) void moe_align_kernel(const int32_t* __restrict__ ids, int n,
                                                         int E, int block,
                                                         int32_t* __restrict__ sorted_ids,
                                                         int32_t* __restrict__ offsets,
                                                         int32_t* __restrict__ num_padded,
                                                         int32_t* __restrict__ inv,
                                                         int32_t* __restrict__ tile_expert,
                                                         int max_tiles) {
  extern __shared__ int sm[];
  int* cnt = sm;             // [E]
  int* cursor = sm + E;      // [E]
  int* offs = sm + 2 * E;    // [E + 1], LDS copy of the padded segment starts
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  // ids outside [0, E) (expert-parallel padding rows) are skipped: no slot, inv = -1
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    if ((unsigned)ids[i] < (unsigned)E) atomicAdd(&cnt[ids[i]], 1);
  __syncthreads();
  if (threadIdx.x == 0) {  // E <= 256 LDS-only adds
    int acc = 0;
    for (int e = 0; e < E; ++e) {
      offs[e] = acc;
      acc += (cnt[e] + block - 1) / block * block;
    }
    offs[E] = acc;
    *num_padded = acc;
  }
  __syncthreads();
  for (int e = threadIdx.x; e <= E; e += blockDim.x) {
    offsets[e] = offs[e];
    if (e < E) cursor[e] = offs[e];
  }
  const int total = offs[E];
  for (int i = threadIdx.x; i < total; i += blockDim.x) sorted_ids[i] = n;
  if (tile_expert != nullptr) {
    // expert of tile t: the last e with offs[e] <= t * block (binary search over LDS; empty
    // experts share their start with the next one, the search lands past them)
    for (int t = threadIdx.x; t < max_tiles; t += blockDim.x) {
      const int r0 = t * block;
      int e = -1;
      if (r0 < total) {
        int lo = 0, hi = E - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (offs[mid] <= r0) lo = mid;
          else hi = mid - 1;
        }
        e = lo;
      }
      tile_expert[t] = e;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    if ((unsigned)ids[i] >= (unsigned)E) {
      if (inv != nullptr) inv[i] = -1;
      continue;
    }
    const int pos = atomicAdd(&cursor[ids[i]], 1);
    sorted_ids[pos] = i;
    if (inv != nullptr) inv[i] = pos;
  }
}

// Grouped GEMM over expert-sorted rows:  Y[r] = A[row(r)] . W[e(tile)]^T
// A_GATHER: row(r) = sorted_ids[r] / topk (token rows of the hidden state; padding rows
// read as zeros); else row(r) = r (the previous grouped GEMM's output).  Same 64x64x64
// MFMA tile as gemm.hip, weights per expert [E, N, K] K-major.
template <bool A_GATHER>
__global__ __launch_bounds__(256) void moe_gemm_kernel(const bf16* __restrict__ A,
                                                       const bf16* __restrict__ W,
                                                       bf16* __restrict__ Y,
                                                       const int32_t* __restrict__ sorted_ids,
                                                       const int32_t* __restrict__ tile_expert,
                                                       int n_flat, int topk, int N, int K,
                                                       int lda) {
  __shared__ bf16x8 lds[2][2][64 * 8];
  const int tile = blockIdx.x;
  const int e = tile_expert[tile];
  if (e < 0) return;  // beyond the padded row count (graph-safe fixed grid)
  const int n0 = blockIdx.y * 64;
  const int m0 = tile * 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int s_row = tid >> 2, s_ch = (tid & 3) * 2;
  int arow;
  bool a_ok;
  if (A_GATHER) {
    const int sid = sorted_ids[m0 + s_row];
    a_ok = sid < n_flat;
    arow = a_ok ? sid / topk : 0;
  } else {
    arow = m0 + s_row;
    a_ok = true;
  }
  const bool b_ok = n0 + s_row < N;
  const bf16* xa = A + (size_t)arow * lda;
  const bf16* wb = W + ((size_t)e * N + (b_ok ? n0 + s_row : 0)) * K;
  const bf16x8 zero8 = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  bf16x8 ra[2], rb[2];
  auto sw = [](int row, int ch) { return row * 8 + (ch ^ (row & 7)); };
  auto gload = [&](int k0) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int kk = k0 + (s_ch + c) * 8;
      ra[c] = (a_ok && kk < K) ? *reinterpret_cast<const bf16x8*>(xa + kk) : zero8;
      rb[c] = (b_ok && kk < K) ? *reinterpret_cast<const bf16x8*>(wb + kk) : zero8;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      lds[buf][0][sw(s_row, s_ch + c)] = ra[c];
      lds[buf][1][sw(s_row, s_ch + c)] = rb[c];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (K + 63) / 64;
  gload(0);
  sstore(0);
  __syncthreads();
  const int fr = lane & 15, fg = lane >> 4;
  for (int it = 0; it < nk; ++it) {
    const int cur = it & 1;
    if (it + 1 < nk) gload((it + 1) * 64);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = lds[cur][0][sw(wm * 32 + i * 16 + fr, ks * 4 + fg)];
        bfr[i] = lds[cur][1][sw(wn * 32 + i * 16 + fr, ks * 4 + fg)];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (it + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 32 + j * 16 + fr;
      if (col >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + i * 16 + fg * 4 + r;
        Y[(size_t)row * N + col] = f2bf(acc[i][j][r]);
      }
    }
}

// out[t] = sum_k w[t,k] * Y[inv[t*K+k]]   (deterministic gather-combine, fp32 sum)
__global__ __launch_bounds__(256) void moe_combine_kernel(const bf16* __restrict__ Y,
                                                          const float* __restrict__ wts,
                                                          const int32_t* __restrict__ inv,
                                                          bf16* __restrict__ out, int T,
                                                          int topk, int d) {
  const int vpr = d / 8;
  const long total = (long)T * vpr;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    // 32-bit split whenever the index fits (total < 2^30 here in practice): a 64-bit
    // division per element is a long software sequence
    int t, c;
    if (total < (1L << 30)) {
      t = (int)i / vpr;
      c = ((int)i - t * vpr) * 8;
    } else {
      t = (int)(i / vpr);
      c = (int)(i % vpr) * 8;
    }
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < topk; ++k) {
      const int pos = inv[(size_t)t * topk + k];
      if (pos < 0) continue;  // skipped (expert-parallel padding) row: contributes nothing
      const float wk = wts[(size_t)t * topk + k];
      const bf16x8 y = *reinterpret_cast<const bf16x8*>(Y + (size_t)pos * d + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += wk * bf2f(y[j]);
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    *reinterpret_cast<bf16x8*>(out + (size_t)t * d + c) = o;
  }
}

void launch_moe_gemm(const void* A, const void* W, void* Y, const int32_t* sorted_ids,
                     const int32_t* tile_expert, int max_tiles, int n_flat, int topk, int N,
                     int K, int lda, int gather, hipStream_t s) {
  if (max_tiles == 0) return;
  dim3 grid(max_tiles, (N + 63) / 64);
  if (gather)
    moe_gemm_kernel<true><<<grid, 256, 0, s>>>((const bf16*)A, (const bf16*)W, (bf16*)Y,
                                               sorted_ids, tile_expert, n_flat, topk, N, K, lda);
  else
    moe_gemm_kernel<false><<<grid, 256, 0, s>>>((const bf16*)A, (const bf16*)W, (bf16*)Y,
                                                sorted_ids, tile_expert, n_flat, topk, N, K, lda);
}

void launch_moe_combine(const void* Y, const float* wts, const int32_t* inv, void* out, int T,
                        int topk, int d, hipStream_t s) {
  if (T == 0) return;
  long blocks = ((long)T * (d / 8) + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  moe_combine_kernel<<<(int)blocks, 256, 0, s>>>((const bf16*)Y, wts, inv, (bf16*)out, T, topk,
                                                 d);
}

void launch_moe_align(const int32_t* topk_ids, int n, int E, int block, int32_t* sorted_ids,
                      int32_t* expert_offsets, int32_t* num_padded, int32_t* inv,
                      int32_t* tile_expert, int max_tiles, hipStream_t s) {
  moe_align_kernel<<<1, 1024, (3 * E + 1) * sizeof(int), s>>>(topk_ids, n, E, block, sorted_ids,
                                                        expert_offsets, num_padded, inv,
                                                        tile_expert, max_tiles);
}

}  // namespace akap
