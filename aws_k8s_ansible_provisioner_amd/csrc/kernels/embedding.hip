// Token-embedding gather for gfx950 (vocab-parallel aware: rows outside
// [vocab_start, vocab_end) produce zeros so a TP all-reduce completes the lookup).
#include "common.h"
#include "kernels.h"

namespace akap {

__global__ __launch_bounds__(256) void embedding_kernel(const int64_t* __restrict__ ids,
                                                        const bf16* __restrict__ table,
                                                        bf16* __restrict__ out, int T, int d,
                                                        int vs, int ve) {
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
    const int64_t id = ids[t];
    bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (id >= vs && id < ve) v = *reinterpret_cast<const bf16x8*>(table + (id - vs) * d + c);
    *reinterpret_cast<bf16x8*>(out + (size_t)t * d + c) = v;
  }
}

// Decode-step prologue in one launch (tp = 1): the embedding row -> residual, residual * ln
// -> a_out (the first layer's input norm, un-normalised: the first projection applies the
// row's rsqrt from ss_out, like every other layer of the fused chain), sum of squares ->
// ss_out, and zbuf[0, zn) zeroed (the chain's per-layer sum-of-squares accumulators).  One
// wave per token; replaces an embedding gather, an RMSNorm and a fill launch.
__global__ __launch_bounds__(256) void embedding_prep_kernel(
    const int64_t* __restrict__ ids, const bf16* __restrict__ table, const bf16* __restrict__ ln,
    bf16* __restrict__ residual, bf16* __restrict__ a_out, float* __restrict__ ss_out,
    float* __restrict__ zbuf, long zn, int T, int d, int vs, int ve) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < zn; i += (long)gridDim.x * 256)
    zbuf[i] = 0.f;
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;  // whole waves
  const int64_t id = ids[t];
  const bool mine = id >= vs && id < ve;
  float ss = 0.f;
  for (int c = lane * 8; c < d; c += 512) {
    bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (mine) v = *reinterpret_cast<const bf16x8*>(table + (id - vs) * d + c);
    const bf16x8 w = *reinterpret_cast<const bf16x8*>(ln + c);
    bf16x8 a;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = bf2f(v[j]);
      ss += x * x;
      a[j] = f2bf(x * bf2f(w[j]));
    }
    *reinterpret_cast<bf16x8*>(residual + (size_t)t * d + c) = v;
    *reinterpret_cast<bf16x8*>(a_out + (size_t)t * d + c) = a;
  }
  ss = wave_sum(ss);
  if (lane == 0) ss_out[t] = ss;
}

void launch_embedding_prep(const int64_t* ids, const void* table, const void* ln, void* residual,
                           void* a_out, float* ss_out, float* zbuf, long zn, int T, int d,
                           int vocab_start, int vocab_end, hipStream_t s) {
  const long need = (T + 3) / 4;
  const long zb = (zn + 255) / 256;
  const long blocks = need > zb ? need : zb;
  if (blocks == 0) return;
  embedding_prep_kernel<<<(int)blocks, 256, 0, s>>>(
      ids, (const bf16*)table, (const bf16*)ln, (bf16*)residual, (bf16*)a_out, ss_out, zbuf, zn,
      T, d, vocab_start, vocab_end);
}

void launch_embedding(const int64_t* ids, const void* table, void* out, int T, int d,
                      int vocab_start, int vocab_end, hipStream_t s) {
  if (T == 0) return;
  long blocks = ((long)T * (d / 8) + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  embedding_kernel<<<(int)blocks, 256, 0, s>>>(ids, (const bf16*)table, (bf16*)out, T, d,
                                               vocab_start, vocab_end);
}

}  // namespace akap
