// Mixture-of-experts routing kernels for gfx950.
//  * moe_topk_softmax: router logits [T, E] -> softmax -> top-k (+ optional renorm).
//    One lane per token (E <= 256 keeps the row in registers/L1).
//  * moe_align: groups the T*K (token, expert) pairs by expert, padding every
//    expert's segment to a multiple of the grouped-GEMM row tile so each tile of
//    the sorted list belongs to exactly one expert.  Single workgroup, LDS counts.
#include "common.h"
#include "kernels.h"

namespace akap {

template <typename T>
__global__ __launch_bounds__(256) void moe_topk_softmax_kernel(const T* __restrict__ logits,
                                                               int ld, int E, int K,
                                                               float* __restrict__ topk_w,
                                                               int32_t* __restrict__ topk_ids,
                                                               int Tn, int renorm) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= Tn) return;
  const T* x = logits + (size_t)t * ld;
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) mx = fmaxf(mx, (float)x[e]);
  float z = 0.f;
  for (int e = 0; e < E; ++e) z += __expf((float)x[e] - mx);
  const float invz = 1.f / z;
  float wsum = 0.f;
  // selection by repeated scan (K is tiny: 1..8); ties -> lowest expert id
  uint64_t taken_lo = 0, taken_hi = 0, taken_2 = 0, taken_3 = 0;
  for (int k = 0; k < K; ++k) {
    float best = -INFINITY;
    int bi = 0;
    for (int e = 0; e < E; ++e) {
      const uint64_t bit = 1ull << (e & 63);
      const uint64_t word = e < 64 ? taken_lo : e < 128 ? taken_hi : e < 192 ? taken_2 : taken_3;
      if (word & bit) continue;
      const float v = (float)x[e];
      if (v > best) { best = v; bi = e; }
    }
    const uint64_t bit = 1ull << (bi & 63);
    if (bi < 64) taken_lo |= bit; else if (bi < 128) taken_hi |= bit;
    else if (bi < 192) taken_2 |= bit; else taken_3 |= bit;
    const float w = __expf(best - mx) * invz;
    topk_w[(size_t)t * K + k] = w;
    topk_ids[(size_t)t * K + k] = bi;
    wsum += w;
  }
  if (renorm) {
    const float inv = 1.f / wsum;
    for (int k = 0; k < K; ++k) topk_w[(size_t)t * K + k] *= inv;
  }
}

void launch_moe_topk_softmax(const void* logits, int ld, int E, int K, float* topk_w,
                             int32_t* topk_ids, int T, int renormalize, hipStream_t s) {
  if (T == 0) return;
  moe_topk_softmax_kernel<bf16><<<(T + 255) / 256, 256, 0, s>>>(
      (const bf16*)logits, ld, E, K, topk_w, topk_ids, T, renormalize);
}

// sorted_ids: [n + E*(block-1)] rounded, filled with n (sentinel) for padding.
__global__ __launch_bounds__(1024) void moe_align_kernel(const int32_t* __restrict__ ids, int n,
                                                         int E, int block,
                                                         int32_t* __restrict__ sorted_ids,
                                                         int32_t* __restrict__ offsets,
                                                         int32_t* __restrict__ num_padded) {
  extern __shared__ int sm[];
  int* cnt = sm;          // [E]
  int* cursor = sm + E;   // [E]
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&cnt[ids[i]], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < E; ++e) {
      offsets[e] = acc;
      cursor[e] = acc;
      acc += (cnt[e] + block - 1) / block * block;
    }
    offsets[E] = acc;
    *num_padded = acc;
  }
  __syncthreads();
  const int total = offsets[E];
  for (int i = threadIdx.x; i < total; i += blockDim.x) sorted_ids[i] = n;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int pos = atomicAdd(&cursor[ids[i]], 1);
    sorted_ids[pos] = i;
  }
}

void launch_moe_align(const int32_t* topk_ids, int n, int E, int block, int32_t* sorted_ids,
                      int32_t* expert_offsets, int32_t* num_padded, hipStream_t s) {
  moe_align_kernel<<<1, 1024, 2 * E * sizeof(int), s>>>(topk_ids, n, E, block, sorted_ids,
                                                        expert_offsets, num_padded);
}

}  // namespace akap
