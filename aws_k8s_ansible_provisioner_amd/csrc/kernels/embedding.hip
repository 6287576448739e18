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

void launch_embedding(const int64_t* ids, const void* table, void* out, int T, int d,
                      int vocab_start, int vocab_end, hipStream_t s) {
  if (T == 0) return;
  long blocks = ((long)T * (d / 8) + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  embedding_kernel<<<(int)blocks, 256, 0, s>>>(ids, (const bf16*)table, (bf16*)out, T, d,
                                               vocab_start, vocab_end);
}

}  // namespace akap
