// Intra-node all-reduce over xGMI peer mappings for the TP decode path.
//
// A TP decode step all-reduces two [B, d] bf16 activations per layer (Llama-3-70B TP=8,
// B=64: 1 MiB); RCCL's ring pays ~2(W-1) link hops of latency for these.  MI355X's xGMI
// mesh is fully connected, so every GPU can read every peer's HBM directly:
//   * one-shot (small messages): each rank stages its input in an IPC-shared buffer,
//     raises a flag on every peer, waits for all peers' flags, then sums all W copies
//     itself -- one exchange, all 7 links busy at once;
//   * two-shot (larger messages): reduce-scatter (rank r sums slice r from all peers into
//     its result buffer) -> flags -> all-gather (read the other slices from the peers).
// Synchronisation is per workgroup: block b of every rank owns the same element chunks,
// so block b only needs block b's flags (no grid-wide barrier).
//
// Ordering argument (every hand-off is {sc0 sc1 stores, sc0 sc1 loads} on both sides, the
// system-scope form of MI355X_MICROARCH.md "Valid forms"; no step relies on a cache
// invalidate or write-back instruction):
//   publish  every handed-off byte (staged input, two-shot partial result) is written by a
//            buffer_store ... sc0 sc1 (write-through: the bytes leave the CU and the XCD's L2
//            for HBM); every storing wave then drains with an explicit `s_waitcnt vmcnt(0)`
//            (inline asm, so no compiler pass can drop it) and reaches the workgroup barrier;
//            only after that barrier does one lane per peer store the epoch into that peer's
//            flag word (a system-scope atomic store, sc0 sc1).
//   consume  one lane per peer polls its flag word with system-scope relaxed atomic loads
//            (sc0 sc1: never served by this CU's L1) until it reads >= the epoch; the waves
//            meet at a barrier behind an `s_waitcnt vmcnt(0)`; then EVERY load of a peer's
//            staged bytes is a buffer_load ... sc0 sc1, which bypasses this CU's L1, and the
//            buffers are hipDeviceMallocUncached (MTYPE UC: no XCD L2 keeps a copy), so no
//            load can return a line cached before the peer's store -- whatever this CU or
//            XCD read in an earlier epoch (tests/test_custom_allreduce_gpu.py pre-reads the
//            peers' lines with plain loads to make any such stale copy present).
//   own data a rank never reads its own staged copy back: its term of the sum comes from
//            its input tensor (written by an earlier kernel on this stream).
//   epochs   per-block counters in device memory, read and written by thread 0 through the
//            vector path (an agent-scope atomic, not s_load: the scalar cache is not kept
//            coherent with vector stores), so a captured launch replays with fresh epochs.
//   reuse    staging / result buffers alternate by epoch parity.  EVERY launch runs all
//            kCarMaxBlocks blocks, and every block advances its epoch and takes part in every
//            flag exchange of the launch (blocks with no vectors of a small message exchange
//            flags only), so all blocks of a rank hold the same epoch = the launch count.  A
//            block writes the parity of epoch e+2 only inside launch e+2; it got there after
//            its own epoch-(e+1) flags from every peer, i.e. after every peer STARTED launch
//            e+1 and so finished ALL blocks of launch e (stream order) -- no peer block can
//            still be reading any epoch-e bytes, whatever index -> block map launch e used.
//            (With a size-dependent grid a block that sat out a small launch lagged its
//            siblings' epoch, and a mixed-kind sequence could restage a region a peer's
//            other block was still reading.)
// Every spin-wait is bounded: on timeout the kernel records an error flag and exits.
//
// Siblings on the same buffers, flags and per-block epochs (so a TP decode hipGraph holds
// only these kernels -- no RCCL call -- and replays across processes that share one GPU as
// well as across the xGMI mesh):
//   all-gather  every rank stages its [R, n] shard (sc0 sc1 stores), one flag exchange, then
//               reads every peer's shard (sc0 sc1 loads) into out[R, W*n] (rank-major column
//               blocks: the vocab-parallel logits);
//   broadcast   the root stages the bytes, one flag exchange, the other ranks read them (the
//               TP decode step's input staging region).
// The reuse argument above needs only that every launch runs the full kCarMaxBlocks grid
// (car_blocks), so it holds for any mix of sizes and kinds (tests/test_custom_allreduce_gpu.py
// runs mixed back-to-back sequences with no host sync).
#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int kCarMaxBlocks = 128;
constexpr int kCarMaxRanks = 8;
constexpr int kCoh = 17;  // buffer op cache bits: sc0 | sc1 (system-coherent)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t car_rsrc(const void* base, const CarArgs& a) {
  // buffer of 4 * half_elems bf16 (staging x2, result x2); the base is wave-uniform (kernarg)
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(a.half_elems * 8), 0x00020000);
}

__device__ __forceinline__ bf16x8 car_ld(__amdgpu_buffer_rsrc_t r, size_t elem) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(elem * 2), 0, kCoh);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ void car_st(__amdgpu_buffer_rsrc_t r, size_t elem, bf16x8 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)(elem * 2), 0,
                                         kCoh);
}

__device__ __forceinline__ bool car_wait(const uint32_t* flag, uint32_t v) {
  // bounded by the constant-rate wall clock (100 MHz on MI3xx): give up after ~2 s
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < v) {
    if (wall_clock64() - t0 > 200000000ull) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// All ranks' blocks `bid` meet at phase `ph` (0 or 1) of epoch ep (see the header).
__device__ __forceinline__ void car_barrier(const CarArgs& a, int bid, uint32_t ep, int ph) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its stores
  __syncthreads();
  const int t = threadIdx.x;
  if (t < a.world) {
    const size_t slot = ((size_t)ph * kCarMaxRanks + a.rank) * kCarMaxBlocks + bid;
    __hip_atomic_store(a.sigs[t] + slot, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const size_t mine = ((size_t)ph * kCarMaxRanks + t) * kCarMaxBlocks + bid;
    if (!car_wait(a.sigs[a.rank] + mine, ep))
      __hip_atomic_fetch_or(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // compiler-only ordering: no peer load may be hoisted above the poll
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

__device__ __forceinline__ uint32_t car_epoch(const CarArgs& a, int bid) {
  __shared__ uint32_t s_ep;
  if (threadIdx.x == 0) {
    const uint32_t ep =
        __hip_atomic_load(a.counter + bid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    __hip_atomic_store(a.counter + bid, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_ep = ep;
  }
  __syncthreads();
  return s_ep;
}

// Store of one reduced 8-vector i: plain, or the residual + next-norm epilogue (CarEpi).
// The epilogue's per-row sum of squares is reduced across the wave first (d % 512 == 0:
// a wave's 64 consecutive vectors lie in one row), then one atomic per wave.
template <bool EPI>
__device__ __forceinline__ void car_store(bf16* __restrict__ out, const CarEpi& e, long i,
                                          const bf16x8& sum) {
  if constexpr (!EPI) {
    reinterpret_cast<bf16x8*>(out)[i] = sum;
  } else {
    const long el = i * 8;
    const int row = (int)(el / e.d), col = (int)(el % e.d);
    bf16x8* rp = reinterpret_cast<bf16x8*>(e.residual) + i;
    const bf16x8 r = *rp;
    const bf16x8 g = *reinterpret_cast<const bf16x8*>(e.ln + col);
    bf16x8 s8, a8;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s8[j] = f2bf(bf2f(sum[j]) + bf2f(r[j]));
      const float f = bf2f(s8[j]);
      a8[j] = f2bf(f * bf2f(g[j]));
      q += f * f;
    }
    *rp = s8;
    reinterpret_cast<bf16x8*>(e.aout)[i] = a8;
    q = wave_sum(q);
    if ((threadIdx.x & 63) == 0) atomicAdd(e.ss + row, q);
  }
}

// Sum of the W ranks' copies of vector i (staged at element offset base + 8i in every peer's
// buffer), in fixed rank order -> identical bits on every rank.  This rank's term is `own`.
__device__ __forceinline__ bf16x8 car_sum(const CarArgs& a, size_t base, long i,
                                          const bf16x8& own) {
  bf16x8 v[kCarMaxRanks];
#pragma unroll
  for (int p = 0; p < kCarMaxRanks; ++p)  // every peer load issued before the first add
    if (p < a.world && p != a.rank) v[p] = car_ld(car_rsrc(a.bufs[p], a), base + (size_t)i * 8);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int p = 0; p < kCarMaxRanks; ++p) {
    if (p >= a.world) break;
    const bf16x8 x = p == a.rank ? own : v[p];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += bf2f(x[j]);
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
  return o;
}

// Test stress (CarMulti::warm): pull the peers' staging lines of this block's vectors into
// this CU's caches with PLAIN loads before the exchange, so a protocol that depended on an
// invalidate would read them stale.  The sink store never happens for finite inputs.
__device__ __forceinline__ void car_prewarm(const CarArgs& a, int bid, int nblk, long n8,
                                            size_t base, bf16* sink) {
  const long stride = (long)nblk * 256;
  float s = 0.f;
  for (long i = (long)bid * 256 + threadIdx.x; i < n8; i += stride)
    for (int p = 0; p < a.world; ++p) {
      const bf16x8 x = reinterpret_cast<const bf16x8*>(a.bufs[p] + base)[i];
      s += bf2f(x[0]);
    }
  if (s == 12345.678f) sink[0] = f2bf(s);
}

// Kernel bodies take the block's identity (bid of nblk) explicitly so the test launcher
// below can run every simulated rank of one process inside one grid.
template <bool EPI>
__device__ __forceinline__ void car_oneshot(const CarArgs& a, int bid, int nblk,
                                            const bf16* __restrict__ in, bf16* __restrict__ out,
                                            long n8, const CarEpi& epi, bool warm) {
  const uint32_t ep = car_epoch(a, bid);
  const size_t par = (ep & 1) * a.half_elems;
  if (warm) car_prewarm(a, bid, nblk, n8, par, out);
  const __amdgpu_buffer_rsrc_t mine = car_rsrc(a.bufs[a.rank], a);
  const bf16x8* src = reinterpret_cast<const bf16x8*>(in);
  const long stride = (long)nblk * 256;
  for (long i = (long)bid * 256 + threadIdx.x; i < n8; i += stride)
    car_st(mine, par + (size_t)i * 8, src[i]);
  car_barrier(a, bid, ep, 0);
  for (long i = (long)bid * 256 + threadIdx.x; i < n8; i += stride)
    car_store<EPI>(out, epi, i, car_sum(a, par, i, src[i]));
}

// Two-shot: n8 split into W slices of s8 vectors (last slice may be short).
template <bool EPI>
__device__ __forceinline__ void car_twoshot(const CarArgs& a, int bid, int nblk,
                                            const bf16* __restrict__ in, bf16* __restrict__ out,
                                            long n8, const CarEpi& epi, bool warm) {
  const uint32_t ep = car_epoch(a, bid);
  const size_t par = (ep & 1) * a.half_elems;
  if (warm) car_prewarm(a, bid, nblk, n8, par, out);
  // staging region: [0, 2*half) input copies by parity; result region: [2*half, 4*half)
  const __amdgpu_buffer_rsrc_t mine = car_rsrc(a.bufs[a.rank], a);
  const bf16x8* src = reinterpret_cast<const bf16x8*>(in);
  const long stride = (long)nblk * 256;
  // slices are whole 64-vector groups: with the epilogue a wave's 64 lanes must stay inside one
  // slice (and so one row, d % 512 == 0) for car_store's wave-wide row sum of squares
  const long s8 = ((n8 + a.world - 1) / a.world + 63) / 64 * 64;
  // staged with the same slice-relative index->block map the reduce uses below, so block
  // b of a peer reads exactly what block b of this rank wrote before its flag (this rank's
  // own slice is not staged: its reduce reads it from `in`)
  for (int p = 0; p < a.world; ++p) {
    if (p == a.rank) continue;
    const long plo = (long)p * s8;
    const long phi = plo + s8 < n8 ? plo + s8 : n8;
    for (long i = plo + (long)bid * 256 + threadIdx.x; i < phi; i += stride)
      car_st(mine, par + (size_t)i * 8, src[i]);
  }
  car_barrier(a, bid, ep, 0);
  const size_t res = 2 * a.half_elems + par;
  // reduce-scatter: my slice [r*s8, min(n8,(r+1)*s8))
  const long lo = (long)a.rank * s8;
  const long hi = lo + s8 < n8 ? lo + s8 : n8;
  for (long i = lo + (long)bid * 256 + threadIdx.x; i < hi; i += stride) {
    const bf16x8 o = car_sum(a, par, i, src[i]);
    car_st(mine, res + (size_t)i * 8, o);
    car_store<EPI>(out, epi, i, o);
  }
  car_barrier(a, bid, ep, 1);
  // all-gather the other slices
  for (int q = 1; q < a.world; ++q) {
    const int p = (a.rank + q) % a.world;
    const long plo = (long)p * s8;
    const long phi = plo + s8 < n8 ? plo + s8 : n8;
    const __amdgpu_buffer_rsrc_t pr = car_rsrc(a.bufs[p], a);
    for (long i = plo + (long)bid * 256 + threadIdx.x; i < phi; i += stride)
      car_store<EPI>(out, epi, i, car_ld(pr, res + (size_t)i * 8));
  }
}

template <bool EPI>
__global__ __launch_bounds__(256) void car_oneshot_kernel(CarArgs a, const bf16* __restrict__ in,
                                                          bf16* __restrict__ out, long n8,
                                                          CarEpi epi) {
  car_oneshot<EPI>(a, blockIdx.x, gridDim.x, in, out, n8, epi, false);
}

template <bool EPI>
__global__ __launch_bounds__(256) void car_twoshot_kernel(CarArgs a, const bf16* __restrict__ in,
                                                          bf16* __restrict__ out, long n8,
                                                          CarEpi epi) {
  car_twoshot<EPI>(a, blockIdx.x, gridDim.x, in, out, n8, epi, false);
}

// Test launcher: blockIdx.y = simulated rank (all ranks' blocks co-resident in one grid).
template <bool EPI>
__global__ __launch_bounds__(256) void car_multi_kernel(CarMulti m, long n8, int two_shot) {
  const int r = blockIdx.y;
  if (two_shot)
    car_twoshot<EPI>(m.args[r], blockIdx.x, gridDim.x, (const bf16*)m.in[r], (bf16*)m.out[r],
                     n8, m.epi[r], m.warm != 0);
  else
    car_oneshot<EPI>(m.args[r], blockIdx.x, gridDim.x, (const bf16*)m.in[r], (bf16*)m.out[r],
                     n8, m.epi[r], m.warm != 0);
}

// All-gather: rank r's shard in[R, n] -> out[R, W*n] columns [r*n, (r+1)*n); n % 8 == 0.
// Each thread moves kCarU vectors per trip (all loads in flight before the stores: one
// vector per thread left a 64-block grid latency-bound at ~1.6 TB/s); staging and reading use
// the same index -> block map, so the per-block flag exchange still covers what it reads.
constexpr int kCarU = 8;

__device__ __forceinline__ void car_allgather(const CarArgs& a, int bid, int nblk,
                                              const bf16* __restrict__ in,
                                              bf16* __restrict__ out, long n8, int n) {
  const uint32_t ep = car_epoch(a, bid);
  const size_t par = (ep & 1) * a.half_elems;
  const __amdgpu_buffer_rsrc_t mine = car_rsrc(a.bufs[a.rank], a);
  const bf16x8* src = reinterpret_cast<const bf16x8*>(in);
  const long step = (long)nblk * 256 * kCarU;
  const long first = (long)bid * 256 * kCarU + threadIdx.x;
  for (long i0 = first; i0 < n8; i0 += step) {
    bf16x8 v[kCarU];
#pragma unroll
    for (int k = 0; k < kCarU; ++k)
      if (i0 + k * 256 < n8) v[k] = src[i0 + k * 256];
#pragma unroll
    for (int k = 0; k < kCarU; ++k)
      if (i0 + k * 256 < n8) car_st(mine, par + (size_t)(i0 + k * 256) * 8, v[k]);
  }
  car_barrier(a, bid, ep, 0);
  const long W = a.world;
  for (long i0 = first; i0 < n8; i0 += step) {
    bf16x8 v[kCarMaxRanks][kCarU];
#pragma unroll
    for (int p = 0; p < kCarMaxRanks; ++p)  // every load in flight before the stores
#pragma unroll
      for (int k = 0; k < kCarU; ++k) {
        const long i = i0 + k * 256;
        if (p < a.world && i < n8)
          v[p][k] = p == a.rank ? src[i] : car_ld(car_rsrc(a.bufs[p], a), par + (size_t)i * 8);
      }
#pragma unroll
    for (int k = 0; k < kCarU; ++k) {
      const long i = i0 + k * 256;
      if (i >= n8) break;
      const long e = i * 8, row = e / n, col = e % n;
      bf16* o = out + row * W * n + col;
#pragma unroll
      for (int p = 0; p < kCarMaxRanks; ++p) {
        if (p >= a.world) break;
        *reinterpret_cast<bf16x8*>(o + (long)p * n) = v[p][k];
      }
    }
  }
}

// Broadcast of n8 16-byte vectors of `buf` from rank `root` to every rank (in place).
__device__ __forceinline__ void car_bcast(const CarArgs& a, int bid, int nblk, bf16* buf,
                                          long n8, int root) {
  const uint32_t ep = car_epoch(a, bid);
  const size_t par = (ep & 1) * a.half_elems;
  const long stride = (long)nblk * 256;
  bf16x8* b8 = reinterpret_cast<bf16x8*>(buf);
  if (a.rank == root) {
    const __amdgpu_buffer_rsrc_t mine = car_rsrc(a.bufs[a.rank], a);
    for (long i = (long)bid * 256 + threadIdx.x; i < n8; i += stride)
      car_st(mine, par + (size_t)i * 8, b8[i]);
  }
  car_barrier(a, bid, ep, 0);
  if (a.rank != root) {
    const __amdgpu_buffer_rsrc_t rr = car_rsrc(a.bufs[root], a);
    for (long i = (long)bid * 256 + threadIdx.x; i < n8; i += stride)
      b8[i] = car_ld(rr, par + (size_t)i * 8);
  }
}

// All-to-all with equal segments: in = [W][seg8 vectors] (segment d goes to rank d), out =
// [W][seg8] with out[p] = rank p's in[rank].  Each block stages, for every destination, the
// same vector indices it later reads from the peers (i in its grid-stride set over seg8), so
// the per-block flag exchange (car_barrier) covers exactly the data each block reads -- the
// ordering argument of the one-shot all-reduce, unchanged.
__device__ __forceinline__ void car_alltoall(const CarArgs& a, int bid, int nblk,
                                             const bf16* __restrict__ in, bf16* __restrict__ out,
                                             long seg8) {
  const uint32_t ep = car_epoch(a, bid);
  const size_t par = (ep & 1) * a.half_elems;
  const __amdgpu_buffer_rsrc_t mine = car_rsrc(a.bufs[a.rank], a);
  const bf16x8* src = reinterpret_cast<const bf16x8*>(in);
  bf16x8* dst = reinterpret_cast<bf16x8*>(out);
  const long step = (long)nblk * 256 * kCarU;
  const long first = (long)bid * 256 * kCarU + threadIdx.x;
  const int W = a.world;
  for (long i0 = first; i0 < seg8; i0 += step)
    for (int d = 0; d < W; ++d) {
      if (d == a.rank) continue;
      bf16x8 v[kCarU];
#pragma unroll
      for (int k = 0; k < kCarU; ++k)
        if (i0 + k * 256 < seg8) v[k] = src[d * seg8 + i0 + k * 256];
#pragma unroll
      for (int k = 0; k < kCarU; ++k)
        if (i0 + k * 256 < seg8) car_st(mine, par + (size_t)(d * seg8 + i0 + k * 256) * 8, v[k]);
    }
  car_barrier(a, bid, ep, 0);
  for (long i0 = first; i0 < seg8; i0 += step) {
    bf16x8 v[kCarMaxRanks][kCarU];
#pragma unroll
    for (int p = 0; p < kCarMaxRanks; ++p)  // every load in flight before the stores
#pragma unroll
      for (int k = 0; k < kCarU; ++k) {
        const long i = i0 + k * 256;
        if (p < W && i < seg8)
          v[p][k] = p == a.rank ? src[a.rank * seg8 + i]
                                : car_ld(car_rsrc(a.bufs[p], a),
                                         par + (size_t)(a.rank * seg8 + i) * 8);
      }
#pragma unroll
    for (int p = 0; p < kCarMaxRanks; ++p) {
      if (p >= W) break;
#pragma unroll
      for (int k = 0; k < kCarU; ++k)
        if (i0 + k * 256 < seg8) dst[p * seg8 + i0 + k * 256] = v[p][k];
    }
  }
}

__global__ __launch_bounds__(256) void car_alltoall_kernel(CarArgs a, const bf16* __restrict__ in,
                                                           bf16* __restrict__ out, long seg8) {
  car_alltoall(a, blockIdx.x, gridDim.x, in, out, seg8);
}

__global__ __launch_bounds__(256) void car_allgather_kernel(CarArgs a, const bf16* __restrict__ in,
                                                            bf16* __restrict__ out, long n8,
                                                            int n) {
  car_allgather(a, blockIdx.x, gridDim.x, in, out, n8, n);
}

__global__ __launch_bounds__(256) void car_bcast_kernel(CarArgs a, bf16* buf, long n8, int root) {
  car_bcast(a, blockIdx.x, gridDim.x, buf, n8, root);
}

// Block count of every launch: the communicator's fixed grid (kCarMaxBlocks by default),
// whatever the size and kind, so every block's epoch counts every launch (header, "reuse").
// Blocks past a small message's vectors only exchange flags.  Ranks that SHARE one GPU (the
// single-GPU rehearsal) use a smaller grid: their spinning blocks otherwise hold a wave slot
// on every SIMD, and a peer's 512-VGPR GEMM workgroup then fits on no CU -- the peer never
// reaches the collective and every wait times out.
static int car_blocks(const CarArgs& a) {
  return a.blocks > 0 && a.blocks <= kCarMaxBlocks ? a.blocks : kCarMaxBlocks;
}

void launch_custom_allreduce(const CarArgs& a, const void* in, void* out, long n, int two_shot,
                             hipStream_t s, const CarEpi* epi) {
  const long n8 = n / 8;
  if (n8 == 0) return;
  const int blocks = car_blocks(a);
  const CarEpi e = epi ? *epi : CarEpi{};
  if (two_shot) {
    if (epi) car_twoshot_kernel<true><<<blocks, 256, 0, s>>>(a, (const bf16*)in, (bf16*)out, n8, e);
    else car_twoshot_kernel<false><<<blocks, 256, 0, s>>>(a, (const bf16*)in, (bf16*)out, n8, e);
  } else {
    if (epi) car_oneshot_kernel<true><<<blocks, 256, 0, s>>>(a, (const bf16*)in, (bf16*)out, n8, e);
    else car_oneshot_kernel<false><<<blocks, 256, 0, s>>>(a, (const bf16*)in, (bf16*)out, n8, e);
  }
}

void launch_custom_allgather(const CarArgs& a, const void* in, void* out, long rows, int n,
                             hipStream_t s) {
  const long n8 = rows * n / 8;
  if (n8 == 0) return;
  car_allgather_kernel<<<car_blocks(a), 256, 0, s>>>(a, (const bf16*)in,
                                                                    (bf16*)out, n8, n);
}

void launch_custom_alltoall(const CarArgs& a, const void* in, void* out, long seg_elems,
                            hipStream_t s) {
  const long seg8 = seg_elems / 8;
  if (seg8 == 0) return;
  car_alltoall_kernel<<<car_blocks(a), 256, 0, s>>>(a, (const bf16*)in,
                                                                      (bf16*)out, seg8);
}

void launch_custom_broadcast(const CarArgs& a, void* buf, long bytes, int root, hipStream_t s) {
  const long n8 = bytes / 16;
  if (n8 == 0) return;
  car_bcast_kernel<<<car_blocks(a), 256, 0, s>>>(a, (bf16*)buf, n8, root);
}

void launch_custom_allreduce_multi(const CarMulti& m, int world, long n, int two_shot,
                                   hipStream_t s) {
  const long n8 = n / 8;
  if (n8 == 0) return;
  dim3 grid(car_blocks(m.args[0]), world);
  if (m.use_epi) car_multi_kernel<true><<<grid, 256, 0, s>>>(m, n8, two_shot);
  else car_multi_kernel<false><<<grid, 256, 0, s>>>(m, n8, two_shot);
}

size_t custom_allreduce_signal_bytes() {
  return (size_t)2 * kCarMaxRanks * kCarMaxBlocks * sizeof(uint32_t);
}

}  // namespace akap
