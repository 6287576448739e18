// KV-cache block pack/unpack for disaggregated prefill/decode on gfx950.
// A sequence's paged blocks (all layers, K and V) are gathered into one contiguous
// buffer so the hand-off is ONE large RCCL send over xGMI instead of L*2*nblk small
// ones, and scattered into the receiver's own block ids on the other side.
// Layout of the packed buffer: [planes][nblk][block_elems].
//
// kv_pull: the hipIpc form of the hand-off (no pack, no send, no unpack).  The prefill
// engine exports its whole KV cache once (hipIpcGetMemHandle); the decode engine maps it
// (hipIpcOpenMemHandle: the same GPU, or a peer over xGMI) and ONE launch copies a batch
// of requests' blocks straight from the peer cache into its own block ids, and fills each
// request's V tail (the token-major partial last 8-token V group the decode attention
// reads, see AttnParams::v_tail) from the same source in the same pass.  Every load of the
// peer's bytes is a buffer_load ... sc0 sc1 (system-coherent: never a line this CU or XCD
// cached earlier -- the blocks are reused by later requests); the producer's plain stores
// were published by its kernels' end-of-kernel release before it announced the blocks
// (the announcing host thread synchronised its stream first).
#include "common.h"
#include "kernels.h"

namespace akap {

template <bool GATHER>
__global__ __launch_bounds__(256) void kv_copy_kernel(bf16* __restrict__ cache, long plane_stride,
                                                      int block_elems,
                                                      const int* __restrict__ block_ids,
                                                      int nblk, int cache_blocks,
                                                      bf16* __restrict__ buf) {
  const int plane = blockIdx.y;
  const int b = blockIdx.x;
  const long src_blk = block_ids[b];
  // the ids are range-checked on the host (KVTransferAgent._ids); this guard keeps a bad id
  // from touching memory past the cache even if a caller skips that check
  if (src_blk < 0 || src_blk >= cache_blocks) return;
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
                      int cache_blocks, const int* block_ids, int nblk, void* out,
                      hipStream_t s) {
  if (nblk == 0) return;
  kv_copy_kernel<true><<<dim3(nblk, planes), 256, 0, s>>>((bf16*)cache, plane_stride, block_elems,
                                                         block_ids, nblk, cache_blocks,
                                                         (bf16*)out);
}

void launch_kv_scatter(const void* in, void* cache, long plane_stride, int planes,
                       int block_elems, int cache_blocks, const int* block_ids, int nblk,
                       hipStream_t s) {
  if (nblk == 0) return;
  kv_copy_kernel<false><<<dim3(nblk, planes), 256, 0, s>>>((bf16*)cache, plane_stride,
                                                          block_elems, block_ids, nblk,
                                                          cache_blocks, (bf16*)in);
}

constexpr int kPullCoh = 17;  // buffer op cache bits: sc0 | sc1 (system-coherent)

__device__ __forceinline__ u32x4 pull_ld(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kPullCoh);
}

// grid.x = nblk * planes copy jobs (then ntail * layers tail jobs).  Copy job j: plane
// j % planes, block pair j / planes -> block_elems bf16 from src_planes[plane][pairs[2b]] to
// dst_planes[plane][pairs[2b+1]].  Tail job: (src block, group, count, slot) x layer l: V-cache
// group [Hkv][D][8] of plane 2l+1 -> tail[l][slot][Hkv][8][D], first `count` tokens.
__global__ __launch_bounds__(256) void kv_pull_kernel(KVPullArgs a) {
  const int job = blockIdx.x;
  const int ncopy = a.nblk * a.planes;
  if (job < ncopy) {
    const int plane = job % a.planes, b = job / a.planes;
    const long sb = a.pairs[2 * b], db = a.pairs[2 * b + 1];
    const bf16* src = reinterpret_cast<const bf16*>(a.src_planes[plane]) + sb * a.block_elems;
    bf16* dst = reinterpret_cast<bf16*>(a.dst_planes[plane]) + db * a.block_elems;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16*>(src), (short)0, a.block_elems * 2, 0x00020000);
    const int nv = a.block_elems / 8;  // 16-byte vectors
    for (int v0 = threadIdx.x; v0 < nv; v0 += 4 * 256) {
      u32x4 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)  // four loads in flight before the first store
        if (v0 + u * 256 < nv) x[u] = pull_ld(r, (v0 + u * 256) * 16);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (v0 + u * 256 < nv) reinterpret_cast<u32x4*>(dst)[v0 + u * 256] = x[u];
    }
    return;
  }
  const int t = job - ncopy;
  const int l = t % a.layers, q = t / a.layers;
  const int sblk = a.tail_jobs[4 * q], grp = a.tail_jobs[4 * q + 1];
  const int cnt = a.tail_jobs[4 * q + 2], slot = a.tail_jobs[4 * q + 3];
  const int D = a.D;
  // V plane 2l+1, block sblk: [Hkv][BS/8][D][8]; this group's [Hkv][D][8] rows
  const bf16* vb = reinterpret_cast<const bf16*>(a.src_planes[2 * l + 1]) +
                   (long)sblk * a.block_elems;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>(vb), (short)0, a.block_elems * 2, 0x00020000);
  bf16* tl = a.tail + ((long)l * a.tail_slots + slot) * a.Hkv * 8 * D;
  for (int i = threadIdx.x; i < a.Hkv * D; i += 256) {  // one (head, dim) row of 8 tokens
    const int h = i / D, d = i % D;
    const long off = ((long)h * (a.BS / 8) + grp) * D * 8 + (long)d * 8;
    const u32x4 w = pull_ld(r, (int)(off * 2));
    const bf16x8 v = __builtin_bit_cast(bf16x8, w);
#pragma unroll
    for (int tt = 0; tt < 8; ++tt)
      if (tt < cnt) tl[((long)h * 8 + tt) * D + d] = v[tt];
  }
}

void launch_kv_pull(const KVPullArgs& a, hipStream_t s) {
  const int jobs = a.nblk * a.planes + a.ntail * a.layers;
  if (jobs == 0) return;
  kv_pull_kernel<<<jobs, 256, 0, s>>>(a);
}

}  // namespace akap
