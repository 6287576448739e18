// Weight warm-up for the decode step: stream the next GEMMs' weights through the cache
// hierarchy (Infinity Cache / MALL) while they are still cold, so the latency-bound
// decode GEMMs that follow read them from MALL instead of HBM.  Loaded words are folded
// into a value that is stored only if impossible, so the loads cannot be eliminated.
#include "common.h"
#include "kernels.h"

namespace akap {

__global__ __launch_bounds__(256) void l2_prefetch_kernel(PrefetchList L, uint32_t* sink) {
  uint32_t acc = 0;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long stride = (long)gridDim.x * 256;
  for (int i = 0; i < L.n; ++i) {
    const u32x4* p = reinterpret_cast<const u32x4*>(L.ptr[i]);
    const long n16 = L.bytes[i] >> 4;
    for (long j = gid; j < n16; j += stride) acc ^= p[j].x;
  }
  if (acc == 0x9E3779B9u && gid == 0) sink[0] = acc;
}

void launch_l2_prefetch(const PrefetchList& L, uint32_t* sink, hipStream_t s) {
  long total = 0;
  for (int i = 0; i < L.n; ++i) total += L.bytes[i];
  if (total == 0) return;
  long blocks = (total / 16 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  l2_prefetch_kernel<<<(int)blocks, 256, 0, s>>>(L, sink);
}

}  // namespace akap
