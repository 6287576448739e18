// KV-cache block pack/unpack for disaggregated prefill/decode on gfx950.
// A sequence's paged blocks (all layers, K and V) are gathered into one contiguous
// buffer so the hand-off is ONE large RCCL send over xGMI instead of L*2*nblk small
// ones, and scattered into the receiver's own block ids on the other side.
// Layout of the packed buffer: [planes][nblk][block_elems].
#include "common.h"
#include "kernels.h"

namespace akap {

template <bool GATHER>
__global__ __launch_bounds__(256) void kv_copy_kernel(bf16* __restrict__ cache, long plane_stride,
                                                      int block_elems,
                                                      const int* __restrict__ block_ids,
                                                      int nblk, bf16* __restrict__ buf) {
  const int plane = blockIdx.y;
  const int b = blockIdx.x;
  const long src_blk = block_ids[b];
  bf16* c = cache + plane * plane_stride + src_blk * block_elems;
  bf16* f = buf + ((long)plane * nblk + b) * block_elems;
  for (int i = threadIdx.x * 8; i < block_elems; i += 256 * 8) {
    if (GATHER)
      *reinterpret_cast<bf16x8*>(f + i) = *reinterpret_cast<const bf16x8*>(c + i);
    else
      *reinterpret_cast<bf16x8*>(c + i) = *reinterpret_cast<const bf16x8*>(f + i);
  }
}

void launch_kv_gather(const void* cache, long plane_stride, int planes, int block_elems,
                      const int* block_ids, int nblk, void* out, hipStream_t s) {
  if (nblk == 0) return;
  kv_copy_kernel<true><<<dim3(nblk, planes), 256, 0, s>>>((bf16*)cache, plane_stride, block_elems,
                                                         block_ids, nblk, (bf16*)out);
}

void launch_kv_scatter(const void* in, void* cache, long plane_stride, int planes,
                       int block_elems, const int* block_ids, int nblk, hipStream_t s) {
  if (nblk == 0) return;
  kv_copy_kernel<false><<<dim3(nblk, planes), 256, 0, s>>>((bf16*)cache, plane_stride,
                                                          block_elems, block_ids, nblk,
                                                          (bf16*)in);
}

}  // namespace akap
