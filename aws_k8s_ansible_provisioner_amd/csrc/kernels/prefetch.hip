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

// In-stream host -> device copy of a step's staging region: the kernel reads the pinned
// (device-mapped) host buffer directly, so the next kernel of the step follows it like any
// kernel -- a hipMemcpyAsync H2D left ~19 us of idle GPU between its copy and the next kernel
// of every decode step (profiles/r4_checkpoint.log step anatomy).  16-B vectors, byte tail.
__global__ __launch_bounds__(256) void h2d_stage_kernel(const uint8_t* __restrict__ src,
                                                        uint8_t* __restrict__ dst, long bytes) {
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long stride = (long)gridDim.x * 256;
  const long n16 = bytes >> 4;
  for (long j = gid; j < n16; j += stride)
    reinterpret_cast<u32x4*>(dst)[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + j);
  for (long j = (n16 << 4) + gid; j < bytes; j += stride) dst[j] = src[j];
}

void launch_h2d_stage(const void* host_src, void* dst, long bytes, hipStream_t s) {
  if (bytes <= 0) return;
  long blocks = ((bytes >> 4) + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 64) blocks = 64;
  h2d_stage_kernel<<<(int)blocks, 256, 0, s>>>((const uint8_t*)host_src, (uint8_t*)dst, bytes);
}

}  // namespace akap
