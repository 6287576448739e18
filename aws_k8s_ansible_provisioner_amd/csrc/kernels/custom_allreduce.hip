// Intra-node all-reduce over xGMI peer mappings for the TP decode path.
//
// A TP decode step all-reduces two [B, d] bf16 activations per layer (Llama-3-70B TP=8,
// B=64: 1 MiB); RCCL's ring pays ~2(W-1) link hops of latency for these.  MI355X's xGMI
// mesh is fully connected, so every GPU can read every peer's HBM directly:
//   * one-shot (small messages): each rank stages its input in an IPC-shared buffer,
//     raises a flag on every peer, waits for all peers' flags, then sums all W staged
//     copies itself -- one exchange, all 7 links busy at once;
//   * two-shot (larger messages): reduce-scatter (rank r sums slice r from all peers into
//     its result buffer) -> flags -> all-gather (read the other slices from the peers).
// Synchronisation is per workgroup: block b of every rank owns the same element chunks,
// so block b only needs block b's flags (no grid-wide barrier).  Flags carry a per-block
// epoch kept in device memory (graph-replay safe: no host-side counter baked into the
// captured launch); staging buffers alternate by epoch parity, so a fast rank never
// overwrites data a slow peer is still reading.  Buffers and flags are allocated
// uncached (hipDeviceMallocUncached) so peer reads never hit stale L2 lines.
// Every spin-wait is bounded: on timeout the kernel records an error flag and exits.
#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int kCarMaxBlocks = 128;
constexpr int kCarMaxRanks = 8;

__device__ __forceinline__ void car_signal(uint32_t* flag, uint32_t v) {
  __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ bool car_wait(const uint32_t* flag, uint32_t v) {
  // bounded by the constant-rate wall clock (100 MHz on MI3xx): give up after ~2 s
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < v) {
    if (wall_clock64() - t0 > 200000000ull) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// All ranks' blocks meet at phase `ph` (0 or 1) of epoch ep.
// Publish: EVERY storing wave drains its own stores with an explicit s_waitcnt AFTER the
// release fence (ROCm 7.2 can drop the fence's own wait -- cdna_hip_programming.md §6
// Guideline 16, Pitfalls 12 and 14: a rare stale peer read under load otherwise) before the
// barrier that lets one lane raise the flags.  Consume: the polling lanes' acquire (buffer_inv)
// is likewise drained before the barrier that releases the other waves' peer loads.
__device__ __forceinline__ void car_barrier(const CarArgs& a, int bid, uint32_t ep, int ph) {
  __threadfence_system();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x;
  const size_t slot = ((size_t)ph * kCarMaxRanks + a.rank) * kCarMaxBlocks + bid;
  if (t < a.world) car_signal(a.sigs[t] + slot, ep);
  if (t < a.world) {
    const size_t mine = ((size_t)ph * kCarMaxRanks + t) * kCarMaxBlocks + bid;
    if (!car_wait(a.sigs[a.rank] + mine, ep)) atomicOr(a.err, 1u);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

__device__ __forceinline__ uint32_t car_epoch(const CarArgs& a, int bid) {
  __shared__ uint32_t s_ep;
  if (threadIdx.x == 0) {
    const uint32_t ep = a.counter[bid] + 1;
    a.counter[bid] = ep;
    s_ep = ep;
  }
  __syncthreads();
  return s_ep;
}

__device__ __forceinline__ void acc_add(float* acc, const bf16x8& v) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
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

// Kernel bodies take the block's identity (bid of nblk) explicitly so the test launcher
// below can run every simulated rank of one process inside one grid.
template <bool EPI>
__device__ __forceinline__ void car_oneshot(const CarArgs& a, int bid, int nblk,
                                            const bf16* __restrict__ in, bf16* __restrict__ out,
                                            long n8, const CarEpi& epi) {
  const uint32_t ep = car_epoch(a, bid);
  const size_t par = (ep & 1) * a.half_elems;
  bf16x8* mine = reinterpret_cast<bf16x8*>(a.bufs[a.rank] + par);
  const bf16x8* src = reinterpret_cast<const bf16x8*>(in);
  const long stride = (long)nblk * 256;
  for (long i = (long)bid * 256 + threadIdx.x; i < n8; i += stride) mine[i] = src[i];
  car_barrier(a, bid, ep, 0);
  bf16x8* dst = reinterpret_cast<bf16x8*>(out);
  for (long i = (long)bid * 256 + threadIdx.x; i < n8; i += stride) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // fixed rank order -> identical result bits on every rank
    for (int p = 0; p < a.world; ++p)
      acc_add(acc, reinterpret_cast<const bf16x8*>(a.bufs[p] + par)[i]);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    car_store<EPI>(out, epi, i, o);
  }
  (void)dst;
}

// Two-shot: n8 split into W slices of s8 vectors (last slice may be short).
template <bool EPI>
__device__ __forceinline__ void car_twoshot(const CarArgs& a, int bid, int nblk,
                                            const bf16* __restrict__ in, bf16* __restrict__ out,
                                            long n8, const CarEpi& epi) {
  const uint32_t ep = car_epoch(a, bid);
  const size_t par = (ep & 1) * a.half_elems;
  // staging region: [0, half) input copies; result region: [2*half, 3*half) by parity
  bf16x8* mine = reinterpret_cast<bf16x8*>(a.bufs[a.rank] + par);
  const bf16x8* src = reinterpret_cast<const bf16x8*>(in);
  const long stride = (long)nblk * 256;
  // slices are whole 64-vector groups: with the epilogue a wave's 64 lanes must stay inside one
  // slice (and so one row, d % 512 == 0) for car_store's wave-wide row sum of squares
  const long s8 = ((n8 + a.world - 1) / a.world + 63) / 64 * 64;
  // staged with the same slice-relative index->block map the reduce uses below, so block
  // b of a peer reads exactly what block b of this rank wrote before its flag
  for (int p = 0; p < a.world; ++p) {
    const long plo = (long)p * s8;
    const long phi = plo + s8 < n8 ? plo + s8 : n8;
    for (long i = plo + (long)bid * 256 + threadIdx.x; i < phi; i += stride)
      mine[i] = src[i];
  }
  car_barrier(a, bid, ep, 0);
  const size_t res = 2 * a.half_elems + par;
  bf16x8* dst = reinterpret_cast<bf16x8*>(out);
  // reduce-scatter: my slice [r*s8, min(n8,(r+1)*s8))
  const long lo = (long)a.rank * s8;
  const long hi = lo + s8 < n8 ? lo + s8 : n8;
  bf16x8* myres = reinterpret_cast<bf16x8*>(a.bufs[a.rank] + res);
  for (long i = lo + (long)bid * 256 + threadIdx.x; i < hi; i += stride) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int p = 0; p < a.world; ++p)
      acc_add(acc, reinterpret_cast<const bf16x8*>(a.bufs[p] + par)[i]);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    myres[i] = o;
    car_store<EPI>(out, epi, i, o);
  }
  car_barrier(a, bid, ep, 1);
  // all-gather the other slices
  for (int q = 1; q < a.world; ++q) {
    const int p = (a.rank + q) % a.world;
    const long plo = (long)p * s8;
    const long phi = plo + s8 < n8 ? plo + s8 : n8;
    const bf16x8* pres = reinterpret_cast<const bf16x8*>(a.bufs[p] + res);
    for (long i = plo + (long)bid * 256 + threadIdx.x; i < phi; i += stride)
      car_store<EPI>(out, epi, i, pres[i]);
  }
  (void)dst;
}

template <bool EPI>
__global__ __launch_bounds__(256) void car_oneshot_kernel(CarArgs a, const bf16* __restrict__ in,
                                                          bf16* __restrict__ out, long n8,
                                                          CarEpi epi) {
  car_oneshot<EPI>(a, blockIdx.x, gridDim.x, in, out, n8, epi);
}

template <bool EPI>
__global__ __launch_bounds__(256) void car_twoshot_kernel(CarArgs a, const bf16* __restrict__ in,
                                                          bf16* __restrict__ out, long n8,
                                                          CarEpi epi) {
  car_twoshot<EPI>(a, blockIdx.x, gridDim.x, in, out, n8, epi);
}

// Test launcher: blockIdx.y = simulated rank (all ranks' blocks co-resident in one grid).
template <bool EPI>
__global__ __launch_bounds__(256) void car_multi_kernel(CarMulti m, long n8, int two_shot) {
  const int r = blockIdx.y;
  if (two_shot)
    car_twoshot<EPI>(m.args[r], blockIdx.x, gridDim.x, (const bf16*)m.in[r], (bf16*)m.out[r],
                     n8, m.epi[r]);
  else
    car_oneshot<EPI>(m.args[r], blockIdx.x, gridDim.x, (const bf16*)m.in[r], (bf16*)m.out[r],
                     n8, m.epi[r]);
}

// Block count for n8 vectors: the same on every rank (a pure function of n8 and world).
static int car_blocks(long n8, int world, bool two) {
  const long per = two ? (n8 + world - 1) / world : n8;
  long b = (per + 255) / 256;
  if (b < 1) b = 1;
  return (int)(b > kCarMaxBlocks ? kCarMaxBlocks : b);
}

void launch_custom_allreduce(const CarArgs& a, const void* in, void* out, long n, int two_shot,
                             hipStream_t s, const CarEpi* epi) {
  const long n8 = n / 8;
  if (n8 == 0) return;
  const int blocks = car_blocks(n8, a.world, two_shot != 0);
  const CarEpi e = epi ? *epi : CarEpi{};
  if (two_shot) {
    if (epi) car_twoshot_kernel<true><<<blocks, 256, 0, s>>>(a, (const bf16*)in, (bf16*)out, n8, e);
    else car_twoshot_kernel<false><<<blocks, 256, 0, s>>>(a, (const bf16*)in, (bf16*)out, n8, e);
  } else {
    if (epi) car_oneshot_kernel<true><<<blocks, 256, 0, s>>>(a, (const bf16*)in, (bf16*)out, n8, e);
    else car_oneshot_kernel<false><<<blocks, 256, 0, s>>>(a, (const bf16*)in, (bf16*)out, n8, e);
  }
}

void launch_custom_allreduce_multi(const CarMulti& m, int world, long n, int two_shot,
                                   hipStream_t s) {
  const long n8 = n / 8;
  if (n8 == 0) return;
  dim3 grid(car_blocks(n8, world, two_shot != 0), world);
  if (m.use_epi) car_multi_kernel<true><<<grid, 256, 0, s>>>(m, n8, two_shot);
  else car_multi_kernel<false><<<grid, 256, 0, s>>>(m, n8, two_shot);
}

size_t custom_allreduce_signal_bytes() {
  return (size_t)2 * kCarMaxRanks * kCarMaxBlocks * sizeof(uint32_t);
}

}  // namespace akap
