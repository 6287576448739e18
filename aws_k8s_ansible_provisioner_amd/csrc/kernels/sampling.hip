// Token sampling for gfx950: greedy, temperature, top-k, top-p over bf16 (or fp32) logits.
//
// Launch structure (launch_sample): ONE sample_chunk_kernel launch, then -- only for batches
// where some row uses top-k / top-p (filtered != 0) -- FOUR sample_pass_kernel launches
// (passes 0..3: histogram passes, a third only when top-p crosses above top-k's bin, and the
// draw); a pass launch whose rows were all resolved earlier returns at once.  Greedy-only batches run argmax_kernel
// instead (one launch).
//   * sample_chunk_kernel: every row is split over chunk workgroups; each publishes an sc1
//     partial record (max, sum of exp, greedy winner, tile masses) and bumps the row's ticket
//     (its own L2 line); the last chunk of a row combines them.  Temperature rows (no filter)
//     are drawn here by INVERSE CDF in three levels -- chunk, then a 2048-element tile from the
//     published tile masses, then one rescan of that tile -- with one exp per element and no
//     per-element RNG.  The chunk kernel also histograms the 256 bf16 keys below each chunk's
//     max: when a row's top-k / top-p threshold falls inside that window it is set exactly here
//     and the row is marked resolved.
//   * sample_pass_kernel: distributed 256-bin histogram passes over the order-preserving
//     16-bit key of the remaining rows find the threshold (by COUNT for top-k, by probability
//     MASS for top-p); the last pass draws a Gumbel-max over the surviving set with a
//     counter-based RNG keyed by (request seed, request step, token id), so a request's stream
//     is reproducible regardless of batch composition.
// No sort anywhere.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace akap {

__device__ __forceinline__ uint32_t fkey(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

struct ArgBest {
  float v;
  int i;
};

__device__ __forceinline__ ArgBest arg_better(ArgBest a, ArgBest b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}

__device__ __forceinline__ ArgBest block_argmax(ArgBest b, float* sv, int* si) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgBest c{__shfl_xor(b.v, o, 64), __shfl_xor(b.i, o, 64)};
    b = arg_better(b, c);
  }
  if (lane == 0) { sv[wid] = b.v; si[wid] = b.i; }
  __syncthreads();
  if (wid == 0) {
    ArgBest c{lane < nw ? sv[lane] : -INFINITY, lane < nw ? si[lane] : 0x7fffffff};
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      ArgBest d{__shfl_xor(c.v, o, 64), __shfl_xor(c.i, o, 64)};
      c = arg_better(c, d);
    }
    if (lane == 0) { sv[0] = c.v; si[0] = c.i; }
  }
  __syncthreads();
  ArgBest r{sv[0], si[0]};
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------------------
// A row of V ~ 152k logits is ~300 KB: one workgroup per row leaves most of the 256 CUs idle
// at decode batch sizes (B = 64 -> 64 CUs) and re-streams the row per pass.
//
// 1. sample_chunk_kernel, grid = (S chunks, B rows; ~512 workgroups, ~1024 with filters): every
//    workgroup streams its chunk with 16-byte loads, 4 in flight per thread, and produces
//      greedy rows   the chunk's argmax (first index on ties);
//      T > 0 rows    per 2048-element tile the (max, sum) of z = x / T, folded into the
//                    chunk's (max, sum) and published tile masses;
//      filtered rows the same plus the chunk's largest logit, then a second visit (from L2)
//                    histograms the 256 bf16 keys below it (pass W, below).
//    The chunk publishes a 32-byte partial record with write-through (sc1) stores and takes
//    a ticket on the row's counter (MI355X_MICROARCH.md "Valid forms", sc1 table row 1: no
//    release / acquire fence -- each costs ~1.7 us and more behind a freshly written logits
//    tensor); the LAST chunk of the row reads the S records with sc1 loads, combines them
//    (max, rescaled sum), re-arms the counter and writes the token + log-prob of a greedy row;
//    a row without filters is drawn there by inverse CDF: u(seed, step) * Z picks the chunk
//    from the prefix of the chunk masses, then the tile from the chunk's published tile
//    masses, then the workgroup rescans that one 2048-element tile (a block scan of
//    per-thread masses) for the token -- exact sampling with one exp per element in the main
//    pass and no per-element RNG; a filtered row's threshold comes from the combined windows
//    when it lies inside them (window_select).
// 2. sample_pass_kernel (passes A-D, grid = (S, B)): thresholds the window could not resolve,
//    by a distributed two-level radix select over the order-preserving 16-bit key -- by COUNT
//    for top-k, by probability MASS for top-p on the top-k renormalised distribution -- then
//    the Gumbel draw over the survivors (details above sample_pass_kernel).
constexpr int kChunkThreads = 256;
constexpr int kMaxChunks = 64;
constexpr int kSc1 = 16;  // buffer op cache bits: sc1 (write-through stores, L1-bypass loads)
constexpr int kSelWords = 16;  // per-row state of the filter passes (32-bit words)
// per-row histogram area of the filter passes, in float2: kMaxChunks x 512 pairs (pass B
// publishes two 256-bin sets per chunk)
constexpr int kHistRow = kMaxChunks * 512;
// draw rows (T > 0, no filter): a chunk is cut into tiles of 2048 consecutive elements (one
// 16-byte vector per thread); the chunk kernel publishes every tile's mass, so the row's last
// chunk rescans ONE tile for the token whatever the chunk size
constexpr int kTile = kChunkThreads * 8;
constexpr int kMaxTiles = 64;  // chunk <= 131072 elements
static_assert((long)kMaxChunks * kMaxTiles * kTile == kSampleMaxVocab, "kernels.h bound");

struct SampPart {  // one chunk's partial record (32 B = two 16-B vectors)
  float m, s;      // max of z over the chunk, sum of exp(z - m)
  float unused0;
  int unused1;
  float am;        // argmax value (greedy rows)
  int ai;
  uint32_t unused2, unused3;
};

template <typename T>
struct Vec;
template <>
struct Vec<bf16> {
  static constexpr int N = 8;
  using type = bf16x8;
};
template <>
struct Vec<float> {
  static constexpr int N = 4;
  using type = f32x4;
};

// Visit x[lo, hi) as f(value, index, ok) with 16-byte loads where the row is aligned.  The
// vector loop issues 4 loads per thread before consuming the oldest: with one load per trip
// every trip paid a full L2 / HBM round trip (load, s_waitcnt vmcnt(0), use), and a chunk
// workgroup's few trips per thread were latency-bound, not bandwidth-bound.  Lanes past the
// range still run f, with ok = false and the value -inf (so a visitor's work and the load
// feeding it stay outside any branch: a load the compiler sinks into a conditional block
// leaves the wait counter unknown, and every later wait becomes vmcnt(0)); visitors that
// count or test keys must honour ok.
template <typename T, typename F>
__device__ __forceinline__ void visit_range(const T* x, int lo, int hi, bool vec_ok, F&& f) {
  constexpr int NV = Vec<T>::N;
  using VT = typename Vec<T>::type;
  if (vec_ok) {
    const int vlo = (lo + NV - 1) / NV, vhi = hi / NV;
    for (int i = lo + threadIdx.x; i < min(hi, vlo * NV); i += blockDim.x) f((float)x[i], i, true);
    const VT* xv = reinterpret_cast<const VT*>(x);
    const int bd = blockDim.x;
    auto use = [&](const VT& q, int v, bool ok) {
#pragma unroll
      for (int j = 0; j < NV; ++j) f(ok ? (float)q[j] : -INFINITY, v * NV + j, ok);
    };
    // batches of 4 unconditional loads (index clamped to the last vector), consumed
    // oldest-first behind counted waits
    if (vlo < vhi) {
      const int last = vhi - 1;
      for (int v = vlo + threadIdx.x; v < vhi; v += 4 * bd) {
        VT q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) q[u] = xv[min(v + u * bd, last)];
#pragma unroll
        for (int u = 0; u < 4; ++u) use(q[u], v + u * bd, v + u * bd < vhi);
      }
    }
    for (int i = max(vhi * NV, vlo * NV) + threadIdx.x; i < hi; i += blockDim.x)
      f((float)x[i], i, true);
  } else {
    for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) f((float)x[i], i, true);
  }
}

// Draw rows' main pass over x[lo, hi): z = x / T in tiles of kTile consecutive elements (8 per
// thread), 4 tiles' loads issued before the first is used (unconditional, index clamped: a
// load under a branch would make every later wait a full drain); per tile a wave-level
// (max, sum exp) pair, then wave 0 folds the pairs into the tile masses (units of exp(z - the
// chunk max)), publishes them to tout with sc1 stores (drained by the caller's ticket wait in
// the same wave) and returns the chunk's (max, sum) to every thread.  XMAX (filtered rows):
// also the chunk's largest logit itself (exact, for the key window) in *xmax.
template <typename T, bool XMAX = false>
__device__ __forceinline__ float2 draw_tiles(const T* x, int lo, int hi, bool vec_ok, float invT,
                                             float* tout, float* xmax = nullptr) {
  __shared__ float2 s_t[kMaxTiles][kChunkThreads / 64];
  __shared__ float2 s_mz;
  __shared__ float s_xm[kChunkThreads / 64];
  float xm = -INFINITY;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n = hi - lo;
  const int ntile = min(kMaxTiles, (n + kTile - 1) / kTile);  // host: chunk <= kMaxTiles tiles
  const int nvf = vec_ok ? n / 8 : 0;  // 8-element groups read as 16-byte vectors
  const T* xc = x + lo;
  float tailx[8];  // the partial last group (vector rows), owned by thread nvf % 256
#pragma unroll
  for (int j = 0; j < 8; ++j) tailx[j] = -INFINITY;
  if (vec_ok && nvf * 8 < n && tid == (nvf & (kChunkThreads - 1)))
    for (int j = 0; j < n - nvf * 8; ++j) tailx[j] = (float)xc[nvf * 8 + j];
  for (int t0 = 0; t0 < ntile; t0 += 4) {
    float z[4][8];
    if (nvf > 0) {  // uniform
      typename Vec<T>::type q[4][8 / Vec<T>::N];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int g = min((t0 + u) * kChunkThreads + tid, nvf - 1);
#pragma unroll
        for (int h = 0; h < 8 / Vec<T>::N; ++h)
          q[u][h] = *reinterpret_cast<const typename Vec<T>::type*>(xc + g * 8 + h * Vec<T>::N);
      }
      // pin all four loads here (the compiler otherwise sinks a load into the lanes that use
      // it, behind a branch, and every wait after that becomes a full drain)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int h = 0; h < 8 / Vec<T>::N; ++h) {
          u32x4 r = __builtin_bit_cast(u32x4, q[u][h]);
          asm volatile("" : "+v"(r));
          q[u][h] = __builtin_bit_cast(typename Vec<T>::type, r);
        }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int g = (t0 + u) * kChunkThreads + tid;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = (float)q[u][j / Vec<T>::N][j % Vec<T>::N];
          const float xv = g < nvf ? v : (g == nvf ? tailx[j] : -INFINITY);
          if constexpr (XMAX) xm = fmaxf(xm, xv);
          z[u][j] = xv * invT;  // -inf stays -inf (invT > 0)
        }
      }
    } else {  // unaligned row (or < 8 elements): scalar loads, index clamped
      float q[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          q[u][j] = (float)xc[min(((t0 + u) * kChunkThreads + tid) * 8 + j, n - 1)];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xv = ((t0 + u) * kChunkThreads + tid) * 8 + j < n ? q[u][j] : -INFINITY;
          if constexpr (XMAX) xm = fmaxf(xm, xv);
          z[u][j] = xv * invT;
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // tiles past ntile (<= 63: t0 <= 60) come out empty
      float mt = -INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) mt = fmaxf(mt, z[u][j]);
      float st = 0.f;
      if (mt > -INFINITY) {
#pragma unroll
        for (int j = 0; j < 8; ++j) st += __expf(z[u][j] - mt);
      }
      const float mw = wave_max_dpp(mt);
      const float sw = wave_sum_dpp(mt == -INFINITY ? 0.f : st * __expf(mt - mw));
      if (lane == 0) s_t[t0 + u][wid] = make_float2(mw, sw);
    }
  }
  if constexpr (XMAX) {
    xm = wave_max_dpp(xm);
    if (lane == 0) s_xm[wid] = xm;
  }
  __syncthreads();
  if constexpr (XMAX) {
    float r = s_xm[0];
#pragma unroll
    for (int w = 1; w < kChunkThreads / 64; ++w) r = fmaxf(r, s_xm[w]);
    *xmax = r;
  }
  if (wid == 0) {
    float mt = -INFINITY, stt = 0.f;
    if (lane < ntile) {
#pragma unroll
      for (int w = 0; w < kChunkThreads / 64; ++w) mt = fmaxf(mt, s_t[lane][w].x);
#pragma unroll
      for (int w = 0; w < kChunkThreads / 64; ++w)
        if (s_t[lane][w].x > -INFINITY) stt += s_t[lane][w].y * __expf(s_t[lane][w].x - mt);
    }
    const float Mc = wave_max(mt);
    const float wl = mt == -INFINITY ? 0.f : stt * __expf(mt - Mc);
    const float Zc = wave_sum(wl);
    const __amdgpu_buffer_rsrc_t rt =
        __builtin_amdgcn_make_buffer_rsrc((void*)tout, (short)0, kMaxTiles * 4, 0x00020000);
    if (lane < ntile) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(wl), rt, lane * 4, 0, kSc1);
    if (lane == 0) s_mz = make_float2(Mc, Zc);
  }
  __syncthreads();
  return s_mz;
}

__device__ __forceinline__ bool row_filtered(const SampleParams& p, int row, float temp) {
  if (!(temp > 0.f)) return false;
  const int k = p.top_k ? p.top_k[row] : 0;
  const float tp = p.top_p ? p.top_p[row] : 1.f;
  return (k > 0 && k < p.V) || (tp < 1.f && tp > 0.f);
}

// state words: 0 M, 1 Z, 2 flags (1 top-k, 2 top-p), 3 sel_hi (pass B bin), 4 cnt_above,
// 5 mass_above, 6 tau (final key threshold, or -1 pending), 7 Zk, 8 p_hi (pass C bin or -1),
// 9 p_above (mass strictly above p_hi's bin inside the top-k set), 10 p_target
struct SelState {
  float M, Z;
  int flags, sel_hi;
  float cnt_above, mass_above;
  int tau;
  float Zk;
  int p_hi;
  float p_above, p_target;
  int kmax16;    // 16-bit key of the row max (chunk kernel)
  int resolved;  // pass W found the threshold inside the window below the max (A-C skip)
  int pad[3];
};
static_assert(sizeof(SelState) == kSelWords * 4, "SelState layout");

__device__ __forceinline__ int k16_of(float v) { return (int)(fkey(v) >> 16); }

// Publish this chunk's NB x 256 (x, y) bins (thread tid holds bins j * 256 + tid) to the row's
// histogram area with sc1 stores, take the row's ticket; in the row's last chunk every thread
// then holds the row totals of its bins in `tot` (the S chunks' loads issued 16 at a time:
// each is a round trip past the per-XCD L2) and true is returned.
template <int NB>
__device__ __forceinline__ bool publish_combine(const float2 (&mine)[NB], float2* hrow, int S,
                                                int c, int* ticket, float2 (&tot)[NB]) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  const int tid = threadIdx.x;
  __shared__ int s_last;
  const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(
      (void*)hrow, (short)0, (int)(S * NB * 256 * 8), 0x00020000);
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    u32x2 v2;
    v2[0] = __float_as_uint(mine[j].x);
    v2[1] = __float_as_uint(mine[j].y);
    __builtin_amdgcn_raw_buffer_store_b64(v2, rh, ((c * NB + j) * 256 + tid) * 8, 0, kSc1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == S - 1;
    if (s_last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return false;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    float tx = 0.f, ty = 0.f;
    for (int q0 = 0; q0 < S; q0 += 16) {
      u32x2 r[16];
#pragma unroll
      for (int k = 0; k < 16; ++k)
        r[k] = __builtin_amdgcn_raw_buffer_load_b64(
            rh, ((min(q0 + k, S - 1) * NB + j) * 256 + tid) * 8, 0, kSc1);
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (q0 + k < S) {
          tx += __uint_as_float(r[k][0]);
          ty += __uint_as_float(r[k][1]);
        }
    }
    tot[j] = make_float2(tx, ty);
  }
  return true;
}

// v = this thread's bin value (bin = threadIdx.x, v >= 0).  Returns the highest bin b with
// sum_{bins >= b} v >= target (bin 0 when even the whole sum stays below; target > 0), and
// sum_{bins > b} v in *above_out.  Every thread calls it (barriers inside).
__device__ __forceinline__ int suffix_select(float v, float target, float* scratch,
                                             float* above_out) {
  __shared__ float s_v[256];
  __shared__ int s_pos;
  __shared__ float s_above;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __syncthreads();  // a previous call's readers are done with s_pos / s_above
  s_v[255 - tid] = v;  // position r holds bin 255 - r: a prefix over positions = a suffix
  if (tid == 0) { s_pos = 255; s_above = 0.f; }
  __syncthreads();
  const float mine = s_v[tid];
  float inc = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) scratch[wid] = inc;
  __syncthreads();
  float before = inc - mine;
  for (int w = 0; w < wid; ++w) before += scratch[w];
  // the unique first position whose inclusive prefix reaches the target (prefixes only grow)
  if (before < target && before + mine >= target) { s_pos = tid; s_above = before; }
  // none reaches it (rounding): bin 0, everything above it
  if (tid == 255 && before + mine < target) s_above = before;
  __syncthreads();
  *above_out = s_above;
  return 255 - s_pos;
}

// Filtered rows, inside the chunk kernel (pass W): the (count, mass) histogram of the 256
// 16-bit keys just below the CHUNK's max key kmc (bin b = key kmc - 255 + b; masses in units
// of exp(z - the chunk's max Mc)), published with sc1 stores to the row's histogram area at
// chunk c.  The row window [km - 255, km] (km = the row max key) is covered: a key of this
// chunk inside it is <= kmc and >= km - 255 >= kmc - 255.  Only in-window elements touch the
// LDS; the chunk was just read, so this second visit comes from L2.
template <typename T>
__device__ __forceinline__ void window_publish(const T* x, int lo, int hi, bool vec_ok,
                                               float invT, float Mc, int kmc, float2* hrow,
                                               int S, int c, bool need_cnt, bool need_mass) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  __shared__ float wl[8 * 256];  // [4 waves][256] counts, then [4 waves][256] masses
  const int tid = threadIdx.x, wid = tid >> 6;
  for (int i = tid; i < 8 * 256; i += kChunkThreads) wl[i] = 0.f;
  __syncthreads();
  const int base = kmc - 255;
  // only the histogram(s) the row's filters read: LDS atomics are this visit's cost (almost
  // every wave has a lane in the window at every element slot); top-k alone counts, top-p
  // alone weighs, top-k + top-p does both
  if (need_cnt && need_mass) {
    visit_range(x, lo, hi, vec_ok, [&](float v, int, bool ok) {
      const int b = k16_of(v) - base;
      if (ok && b >= 0 && b < 256) {
        atomicAdd(&wl[wid * 256 + b], 1.f);
        atomicAdd(&wl[1024 + wid * 256 + b], __expf(v * invT - Mc));
      }
    });
  } else if (need_cnt) {
    visit_range(x, lo, hi, vec_ok, [&](float v, int, bool ok) {
      const int b = k16_of(v) - base;
      if (ok && b >= 0 && b < 256) atomicAdd(&wl[wid * 256 + b], 1.f);
    });
  } else {
    visit_range(x, lo, hi, vec_ok, [&](float v, int, bool ok) {
      const int b = k16_of(v) - base;
      if (ok && b >= 0 && b < 256) atomicAdd(&wl[1024 + wid * 256 + b], __expf(v * invT - Mc));
    });
  }
  __syncthreads();
  float cc = 0.f, mm = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    cc += wl[w * 256 + tid];
    mm += wl[1024 + w * 256 + tid];
  }
  const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(
      (void*)hrow, (short)0, (int)(S * 256 * 8), 0x00020000);
  u32x2 v2;
  v2[0] = __float_as_uint(cc);
  v2[1] = __float_as_uint(mm);
  __builtin_amdgcn_raw_buffer_store_b64(v2, rh, (c * 256 + tid) * 8, 0, kSc1);
  // (drained together with the chunk record, before the row ticket)
}

// The row's last chunk: sum the S chunk windows shifted onto the row window (bin b = key
// km - 255 + b; masses rescaled to exp(z - Mr)), then select.  Resolved when the threshold
// lies inside the window: top-k by count (the window holds >= k elements), top-p by mass
// (the window holds >= the target mass, with a margin over the rounding of two summation
// orders), top-k + top-p as top-p over the top-k set (inside the window with it).  Every
// thread calls it (tid = bin); thread 0 writes the row's SelState.
__device__ __forceinline__ void window_select(const SampleParams& p, int row, SelState& rs,
                                              const float2* hrow, int S, int km, float Mr,
                                              float Zr, const int* ckm, const float* crm) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  __shared__ float scratch[16];
  const int tid = threadIdx.x;
  const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(
      (void*)hrow, (short)0, (int)(S * 256 * 8), 0x00020000);
  float cnt = 0.f, mass = 0.f;
  for (int q0 = 0; q0 < S; q0 += 16) {
    u32x2 r[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int q = min(q0 + k, S - 1);
      const int off = min(255, tid + (km - ckm[q]));
      r[k] = __builtin_amdgcn_raw_buffer_load_b64(rh, (q * 256 + off) * 8, 0, kSc1);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int q = q0 + k;
      if (q < S && tid + (km - ckm[q]) <= 255 && crm[q] > -INFINITY) {
        cnt += __uint_as_float(r[k][0]);
        mass += __uint_as_float(r[k][1]) * __expf(crm[q] - Mr);
      }
    }
  }
  const int kk = p.top_k ? p.top_k[row] : 0;
  const float tp = p.top_p ? p.top_p[row] : 1.f;
  const bool has_k = kk > 0 && kk < p.V, has_p = tp < 1.f && tp > 0.f;
  const int base = km - 255;
  int tau = -1;
  float above, Zk = 0.f;
  if (has_k) {
    if (block_sum(cnt, scratch) >= (float)kk) {  // integer counts: exact
      const int bk = suffix_select(cnt, (float)kk, scratch, &above);
      if (!has_p) {
        tau = base + bk;
      } else {  // top-p over the top-k set, which lies inside the window
        const float mk = tid >= bk ? mass : 0.f;
        Zk = block_sum(mk, scratch);
        const int bp = suffix_select(mk, tp * Zk, scratch, &above);
        tau = base + max(bk, bp);
      }
    }
  } else {
    const float target = tp * Zr;
    if (block_sum(mass, scratch) >= target * 1.0001f)
      tau = base + suffix_select(mass, target, scratch, &above);
  }
  if (tid == 0) {
    rs.M = Mr;
    rs.Z = Zr;
    rs.kmax16 = km;
    rs.tau = tau;
    rs.Zk = Zk;
    rs.p_hi = -1;
    rs.resolved = tau >= 0 ? 1 : 0;
  }
}

template <typename T>
__global__ __launch_bounds__(kChunkThreads) void sample_chunk_kernel(SampleParams p, SampPart* ws,
                                                                     int* tickets, float* rowsum,
                                                                     float* tiles, float2* hist) {
  __shared__ float sv[16];
  __shared__ int si[16];
  __shared__ int s_last;
  const int row = blockIdx.y, c = blockIdx.x, S = gridDim.x;
  const T* x = reinterpret_cast<const T*>(p.logits) + (size_t)row * p.ld;
  const int V = p.V;
  const bool vec_ok = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  constexpr int NV = Vec<T>::N;
  const int chunk = ((V + S - 1) / S + NV - 1) / NV * NV;
  const int lo = min(V, c * chunk), hi = min(V, lo + chunk);
  const float temp = p.temperature ? p.temperature[row] : 0.f;
  const bool greedy = !(temp > 0.f);
  const bool filt = row_filtered(p, row, temp);
  const float invT = greedy ? 1.f : 1.f / temp;
  const bool need_sum = !greedy || (p.greedy_logprobs && p.out_logprobs);
  const uint64_t seed = p.seeds ? (uint64_t)p.seeds[row] : 0x1234ull + row;
  const uint32_t step = p.steps ? (uint32_t)p.steps[row] : 0u;

  // ---- one pass over the chunk (the three row kinds as separate loops: no per-element
  // branch on the row kind) ----
  float m = -INFINITY, sum = 0.f;
  float2 dmz = make_float2(-INFINITY, 0.f);
  ArgBest best{-INFINITY, 0x7fffffff};
  if (!need_sum) {
    visit_range(x, lo, hi, vec_ok, [&](float v, int i, bool) {
      if (v > best.v) { best.v = v; best.i = i; }  // ascending i per thread: first max kept
    });
  } else if (!greedy && !filt) {
    dmz = draw_tiles(x, lo, hi, vec_ok, invT,
                     tiles + ((size_t)row * kMaxChunks + c) * kMaxTiles);
  } else if (filt) {  // (M, Z) as a draw row (its tile masses go unused) + the largest logit
    dmz = draw_tiles<T, true>(x, lo, hi, vec_ok, invT,
                              tiles + ((size_t)row * kMaxChunks + c) * kMaxTiles, &best.v);
  } else {  // greedy with log-probs
    visit_range(x, lo, hi, vec_ok, [&](float v, int i, bool) {
      if (v > best.v) { best.v = v; best.i = i; }
      const float z = v * invT;
      if (z > m) { sum = sum * __expf(m - z) + 1.f; m = z; }
      else if (z > -INFINITY) sum += __expf(z - m);
    });
  }
  // workgroup reductions
  const bool draw = !greedy && !filt;  // uniform over the workgroup
  if (!need_sum || greedy) best = block_argmax(best, sv, si);
  float M = -INFINITY, Z = 0.f;
  if (draw || filt) {
    M = dmz.x;
    Z = dmz.y;
  } else if (need_sum) {
    M = block_max(m, sv);
    Z = block_sum(m == -INFINITY ? 0.f : sum * __expf(m - M), sv);
  }
  // filtered rows: the window histogram below this chunk's max (pass W, first half)
  float2* hrow = hist + (size_t)row * kHistRow;
  int kmc = 0;
  if (filt) {
    kmc = k16_of(best.v);
    const int kk = p.top_k ? p.top_k[row] : 0;
    window_publish(x, lo, hi, vec_ok, invT, M, kmc, hrow, S, c, kk > 0 && kk < V,
                   p.top_p && p.top_p[row] < 1.f && p.top_p[row] > 0.f);
  }
  // ---- publish the partial (sc1 stores), take a ticket ----
  const __amdgpu_buffer_rsrc_t rws = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(ws + (size_t)row * S), (short)0, (int)(S * sizeof(SampPart)), 0x00020000);
  if (threadIdx.x == 0) {
    u32x4 a, b2;
    a[0] = __float_as_uint(M); a[1] = __float_as_uint(Z);
    a[2] = 0u; a[3] = 0u;
    b2[0] = __float_as_uint(best.v); b2[1] = (uint32_t)best.i; b2[2] = (uint32_t)kmc; b2[3] = 0u;
    __builtin_amdgcn_raw_buffer_store_b128(a, rws, c * 32, 0, kSc1);
    __builtin_amdgcn_raw_buffer_store_b128(b2, rws, c * 32 + 16, 0, kSc1);
  }
  if (filt) {  // every wave's window stores drain before the ticket (one round trip with the
               // record's)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int t = __hip_atomic_fetch_add(tickets + row * kCtrStride, 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == S - 1;
  }
  __syncthreads();
  if (!s_last) return;
  // ---- last chunk of the row: combine the S partials (S <= 64: wave 0, sc1 loads) ----
  __shared__ float s_m, s_z, s_res;
  __shared__ int s_chunk, s_tile, s_tok, s_fb, s_km;
  __shared__ int s_ckm[kMaxChunks];
  __shared__ float s_crm[kMaxChunks];
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    float rm = -INFINITY, rs = 0.f;
    ArgBest a{-INFINITY, 0x7fffffff};
    if (l < S) {
      const u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(rws, l * 32, 0, kSc1);
      const u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(rws, l * 32 + 16, 0, kSc1);
      rm = __uint_as_float(v0[0]); rs = __uint_as_float(v0[1]);
      a = ArgBest{__uint_as_float(v1[0]), (int)v1[1]};
      s_ckm[l] = (int)v1[2];
      s_crm[l] = rm;
    }
    const float Mr = wave_max(rm);
    // chunk l's mass in units of exp(z - Mr); its inclusive prefix over the chunks
    const float w = rm == -INFINITY ? 0.f : rs * __expf(rm - Mr);
    float incl = w;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float u = __shfl_up(incl, o, 64);
      if (l >= o) incl += u;
    }
    const float Zr = __shfl(incl, 63, 64);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      ArgBest ca{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64)};
      a = arg_better(a, ca);
    }
    if (draw) {
      // inverse CDF, level 1: the chunk whose prefix mass first reaches u * Z
      const float target = uniform01(seed, step, 0xffffffffu) * Zr;
      const uint64_t hit = __ballot(incl >= target && w > 0.f);
      const uint64_t live = __ballot(w > 0.f);
      // (no live chunk: every logit -inf -- chunk 0, whose tiles are empty too)
      const int c_sel = hit ? __builtin_ctzll(hit) : (live ? 63 - __builtin_clzll(live) : 0);
      // level 1.5: the tile inside that chunk, from its published tile masses (each in
      // units of exp(z - the chunk's max))
      const float r1 = __shfl(hit ? target - (incl - w) : w, c_sel, 64);  // rounding: last mass
      const float scale = __expf(__shfl(rm, c_sel, 64) - Mr);
      const int chunk_len = min(V, (c_sel + 1) * chunk) - min(V, c_sel * chunk);
      const int ntile = (chunk_len + kTile - 1) / kTile;
      const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(tiles + ((size_t)row * kMaxChunks + c_sel) * kMaxTiles), (short)0,
          kMaxTiles * 4, 0x00020000);
      const float tw = l < ntile ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                                       rt, l * 4, 0, kSc1)) * scale
                                 : 0.f;
      float tinc = tw;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float u = __shfl_up(tinc, o, 64);
        if (l >= o) tinc += u;
      }
      const uint64_t thit = __ballot(tinc >= r1 && tw > 0.f);
      const uint64_t tlive = __ballot(tw > 0.f);
      const int t_sel = thit ? __builtin_ctzll(thit) : (tlive ? 63 - __builtin_clzll(tlive) : 0);
      if (l == t_sel) s_res = thit ? r1 - (tinc - tw) : tw;
      if (l == 0) {
        s_chunk = c_sel;
        s_tile = t_sel;
        if (!tlive) s_res = 0.f;
        s_m = Mr;
        s_z = Zr;
        s_tok = 0x7fffffff;
        s_fb = -1;
      }
    }
    if (l == 0) {
      __hip_atomic_store(tickets + row * kCtrStride, 0, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);  // re-arm
      if (greedy) {
        p.out_tokens[row] = a.i;
        // greedy log-prob: x[tok] is the max, so log softmax = -log sum exp(x - M)
        if (p.out_logprobs) p.out_logprobs[row] = p.greedy_logprobs ? -__logf(Zr) : 0.f;
      } else if (filt) {  // window_select below, then the filter passes, finish the row
        s_m = Mr;
        s_z = Zr;
        s_km = k16_of(a.v);
      }
      // rows without filters: passes A-C return at once (their first read)
      if (!filt) reinterpret_cast<SelState*>(rowsum)[row].resolved = 1;
    }
  }
  if (filt) {
    __syncthreads();
    window_select(p, row, reinterpret_cast<SelState*>(rowsum)[row], hrow, S, s_km, s_m, s_z,
                  s_ckm, s_crm);
    return;
  }
  if (!draw) return;
  __syncthreads();
  // ---- inverse CDF, level 2: rescan the selected tile (read by this row's chunk kernel,
  // so in L2), 8 elements per thread; a block scan of the per-thread masses finds the thread
  // whose 8 elements cross the residual mass, which walks them ----
  const float Mr = s_m;
  float R = s_res;
  const int clo = min(V, s_chunk * chunk), chi = min(V, clo + chunk);
  const int lo2 = min(chi, clo + s_tile * kTile), hi2 = min(chi, lo2 + kTile);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int TILE = kTile;
  for (int t0 = lo2; t0 < hi2; t0 += TILE) {
    const int a0 = t0 + (int)threadIdx.x * 8, a1 = min(hi2, a0 + 8);
    float e[8];
    float ts = 0.f;
    int last_pos = -1;
    float xv8[8];
    if (vec_ok && a0 + 8 <= a1) {
      const typename Vec<T>::type q0 = *reinterpret_cast<const typename Vec<T>::type*>(x + a0);
      if constexpr (NV == 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) xv8[j] = (float)q0[j];
      } else {
        const typename Vec<T>::type q1 =
            *reinterpret_cast<const typename Vec<T>::type*>(x + a0 + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { xv8[j] = (float)q0[j]; xv8[4 + j] = (float)q1[j]; }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) xv8[j] = a0 + j < a1 ? (float)x[a0 + j] : -INFINITY;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      e[j] = a0 + j < a1 ? __expf(xv8[j] * invT - Mr) : 0.f;
      ts += e[j];
      if (e[j] > 0.f) last_pos = a0 + j;
    }
    float inc = ts;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    if (lane == 63) sv[wid] = inc;
    __syncthreads();
    float before = inc - ts, total = 0.f;
    for (int wv = 0; wv < kChunkThreads / 64; ++wv) {
      if (wv < wid) before += sv[wv];
      total += sv[wv];
    }
    if (last_pos >= 0) atomicMax(&s_fb, last_pos);
    if (ts > 0.f && R >= before && R < before + ts) {
      float acc = before;
      int tok = last_pos;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc += e[j];
        if (acc > R) { tok = a0 + j; break; }
      }
      atomicMin(&s_tok, tok);
    }
    __syncthreads();
    if (s_tok != 0x7fffffff) break;  // uniform: found in this tile
    R -= total;
  }
  if (threadIdx.x == 0) {
    int tok = s_tok != 0x7fffffff ? s_tok : s_fb;  // rounding past the chunk's end: last mass
    if (tok < 0 || tok >= V) tok = 0;
    p.out_tokens[row] = tok;
    if (p.out_logprobs) p.out_logprobs[row] = (float)x[tok] * invT - Mr - __logf(s_z);
  }
}

// ---------------------------------------------------------------------------------------
// Rows with top-k / top-p: exact thresholds on the 16-bit order-preserving key of the logit
// (k16 = fkey(x) >> 16: exact for bf16 logits, the top 16 bits of an fp32 logit), found by two
// 256-bin histogram levels -- the key's high byte, then its low byte inside the selected
// high-byte bin -- each pass spread over the row's S chunk workgroups like the chunk kernel:
// per-wave LDS histograms, 256 (count, mass) pairs published per chunk with sc1 stores, a
// ticket, and the row's last chunk sums the S histograms and selects (masses are
// exp(x / T - M) with the row max M of the chunk kernel, so they add across chunks).
//   pass W  (in the chunk kernel) (count, mass) histogram of the 256 keys just below the max:
//           when the top-k / top-p threshold falls inside that window (any peaked
//           distribution, and top-k for small k) the exact threshold comes out there -- only
//           in-window elements touch the LDS -- and passes A-C return at once for the row
//           (one read each; folding B and C into A's last chunk saved ~4 us per call but made
//           unresolved rows 2-3x slower: profiles/r5_sampler_rework_2.md);
//   pass A  high-byte histogram of the whole row -> top-k's high byte (by count) or, for a
//           top-p-only row, top-p's high byte (by mass);
//   pass B  low-byte histogram inside that bin -> the exact top-k key (and Zk, the top-k mass)
//           or the exact top-p key; top-k + top-p: top-p over the top-k set, whose crossing is
//           either inside top-k's bin (exact now) or in a higher high-byte bin (pass C);
//   pass C  low-byte mass histogram of that higher bin -> the exact top-p key;
//   pass D  Gumbel-max draw over {k16 >= tau} (RNG only for survivors), best per chunk, the
//           last chunk picks the row's token.
// Every pass reads the row once in parallel (from L2 / MALL after the chunk kernel); rows
// without filters leave every pass at once, and a batch with no filtered row launches none
// of them (ops.sample(filtered=False)).
template <typename T, bool PASS_A>
__global__ __launch_bounds__(kChunkThreads) void sample_pass_kernel(SampleParams p, int pass,
                                                                    SelState* st, float2* hist,
                                                                    int* tickets) {
  // pass A: a per-LANE copy of the high-byte histogram ([bin][lane], 64 KB): a wave's 64
  // lanes never add to the same word (logits crowd into a few exponent bins, and same-word
  // LDS atomics inside one instruction serialise); passes B / C: per-wave histograms of the
  // few elements inside one high-byte bin (and, for top-k + top-p, above it)
  __shared__ float lds[PASS_A ? 256 * 64 : 12 * 256];  // 64 KB only for pass A's lane copies
  __shared__ float scratch[16];
  const int row = blockIdx.y, c = blockIdx.x, S = gridDim.x;
  SelState& rs = st[row];
  // A-C: rows without filters, and filtered rows the window pass resolved (one read)
  if (pass < 3 && rs.resolved) return;
  const float temp = p.temperature ? p.temperature[row] : 0.f;
  if (!row_filtered(p, row, temp)) return;  // uniform
  const T* x = reinterpret_cast<const T*>(p.logits) + (size_t)row * p.ld;
  const int V = p.V;
  const bool vec_ok = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  constexpr int NV = Vec<T>::N;
  const int chunk = ((V + S - 1) / S + NV - 1) / NV * NV;
  const int lo = min(V, c * chunk), hi = min(V, lo + chunk);
  const float invT = 1.f / temp;
  const float M = rs.M;
  int* ticket = tickets + row * kCtrStride;
  float2* hrow = hist + (size_t)row * kHistRow;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kk = p.top_k ? p.top_k[row] : 0;
  const float tp = p.top_p ? p.top_p[row] : 1.f;
  const bool has_k = kk > 0 && kk < V, has_p = tp < 1.f && tp > 0.f;
  if constexpr (PASS_A) {  // A: high byte of the whole row; count (top-k) or mass (top-p only)
    for (int i = tid; i < 256 * 64; i += kChunkThreads) lds[i] = 0.f;
    __syncthreads();
    if (has_k) {
      visit_range(x, lo, hi, vec_ok, [&](float v, int, bool ok) {
        atomicAdd(&lds[(k16_of(v) >> 8) * 64 + lane], ok ? 1.f : 0.f);
      });
    } else {
      visit_range(x, lo, hi, vec_ok, [&](float v, int, bool) {  // -inf: mass 0
        atomicAdd(&lds[(k16_of(v) >> 8) * 64 + lane], __expf(v * invT - M));
      });
    }
    __syncthreads();
    float v = 0.f;  // bin tid over the 64 lane copies (rotated: conflict-free)
#pragma unroll 8
    for (int j = 0; j < 64; ++j) v += lds[tid * 64 + ((j + lane) & 63)];
    float2 mine[1] = {make_float2(v, 0.f)}, tot[1];
    if (!publish_combine<1>(mine, hrow, S, c, ticket, tot)) return;
    float above;
    const int b = suffix_select(tot[0].x, has_k ? (float)kk : tp * rs.Z, scratch, &above);
    if (tid == 0) {
      rs.sel_hi = b;
      if (has_k) rs.cnt_above = above;
      else { rs.mass_above = above; rs.p_target = tp * rs.Z; }
      rs.tau = -1;
      rs.p_hi = -1;
    }
    return;
  } else {
  if (pass == 1) {  // B: low byte inside sel_hi (count + mass); top-k + top-p: masses above
    const int sh = rs.sel_hi;
    float* lc = lds;             // [4][256] low-byte counts
    float* lm = lds + 4 * 256;   // [4][256] low-byte masses
    float* hm = lds + 8 * 256;   // [4][256] high-byte masses of bins above sh
    for (int i = tid; i < 12 * 256; i += kChunkThreads) lds[i] = 0.f;
    __syncthreads();
    const bool above_too = has_k && has_p;
    visit_range(x, lo, hi, vec_ok, [&](float v, int, bool ok) {
      const int k = k16_of(v), h = k >> 8;
      if (!ok) return;
      if (h == sh) {
        atomicAdd(&lc[wid * 256 + (k & 255)], 1.f);
        atomicAdd(&lm[wid * 256 + (k & 255)], __expf(v * invT - M));
      } else if (above_too && h > sh) {
        atomicAdd(&hm[wid * 256 + h], __expf(v * invT - M));
      }
    });
    __syncthreads();
    float cc = 0.f, mm = 0.f, hh = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      cc += lc[w * 256 + tid];
      mm += lm[w * 256 + tid];
      hh += hm[w * 256 + tid];
    }
    float2 mine[2] = {make_float2(cc, mm), make_float2(hh, 0.f)}, tot[2];
    if (!publish_combine<2>(mine, hrow, S, c, ticket, tot)) return;
    const float cnt = tot[0].x, mass = tot[0].y, hmass = tot[1].x;
    float above;
    if (has_k) {
      const int b = suffix_select(cnt, (float)kk - rs.cnt_above, scratch, &above);
      const int tau_k = (sh << 8) | b;
      if (!has_p) {
        if (tid == 0) rs.tau = tau_k;
        return;
      }
      // top-p over the top-k set: Zk = masses of the high-byte bins above sh + low bins >= b
      const float hsum = block_sum(hmass, scratch);
      const float Zk = hsum + block_sum(tid >= b ? mass : 0.f, scratch);
      const float target = tp * Zk;
      if (hsum >= target) {  // crossing in a higher high-byte bin: pass C resolves it
        float habove;
        const int hb = suffix_select(hmass, target, scratch, &habove);
        if (tid == 0) { rs.p_hi = hb; rs.p_above = habove; rs.p_target = target; rs.tau = tau_k; }
        return;
      }
      float lab;
      const int lb = suffix_select(tid >= b ? mass : 0.f, target - hsum, scratch, &lab);
      if (tid == 0) { rs.tau = max(tau_k, (sh << 8) | lb); rs.Zk = Zk; }
      return;
    }
    const int b = suffix_select(mass, rs.p_target - rs.mass_above, scratch, &above);
    if (tid == 0) rs.tau = (sh << 8) | b;
    return;
  }
  if (pass == 2) {  // C: low-byte masses inside p_hi (top-k + top-p rows crossing above sh)
    const int ph = rs.p_hi;
    if (ph < 0) return;  // uniform per row
    float* lm = lds;
    for (int i = tid; i < 4 * 256; i += kChunkThreads) lds[i] = 0.f;
    __syncthreads();
    visit_range(x, lo, hi, vec_ok, [&](float v, int, bool ok) {
      const int k = k16_of(v);
      if (ok && (k >> 8) == ph) atomicAdd(&lm[wid * 256 + (k & 255)], __expf(v * invT - M));
    });
    __syncthreads();
    float mm = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) mm += lm[w * 256 + tid];
    float2 mine[1] = {make_float2(mm, 0.f)}, tot[1];
    if (!publish_combine<1>(mine, hrow, S, c, ticket, tot)) return;
    float above;
    const int b = suffix_select(tot[0].x, rs.p_target - rs.p_above, scratch, &above);
    if (tid == 0) { rs.tau = (ph << 8) | b; rs.p_hi = -1; }
    return;
  }
  // D: Gumbel-max draw over the survivors
  const int tau = rs.tau;
  const uint64_t seed = p.seeds ? (uint64_t)p.seeds[row] : 0x1234ull + row;
  const uint32_t step = p.steps ? (uint32_t)p.steps[row] : 0u;
  ArgBest b{-INFINITY, 0x7fffffff};
  visit_range(x, lo, hi, vec_ok, [&](float v, int i, bool ok) {
    if (!ok || k16_of(v) < tau) return;
    const float u = uniform01(seed, step, (uint32_t)i);
    const float g = v * invT - __logf(-__logf(u));
    if (g > b.v) { b.v = g; b.i = i; }
  });
  __shared__ float sv[16];
  __shared__ int si[16];
  b = block_argmax(b, sv, si);
  __shared__ int s_last;
  const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(
      (void*)hrow, (short)0, (int)(S * 8), 0x00020000);
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  if (tid == 0) {
    u32x2 v2;
    v2[0] = __float_as_uint(b.v);
    v2[1] = (uint32_t)b.i;
    __builtin_amdgcn_raw_buffer_store_b64(v2, rh, c * 8, 0, kSc1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == S - 1;
    if (s_last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last || tid >= 64) return;
  ArgBest a{-INFINITY, 0x7fffffff};
  if (tid < S) {
    const u32x2 r = __builtin_amdgcn_raw_buffer_load_b64(rh, tid * 8, 0, kSc1);
    a = ArgBest{__uint_as_float(r[0]), (int)r[1]};
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgBest ca{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64)};
    a = arg_better(a, ca);
  }
  if (tid == 0) {
    int tok = a.i;
    if (tok < 0 || tok >= V) tok = 0;
    p.out_tokens[row] = tok;
    if (p.out_logprobs) p.out_logprobs[row] = (float)x[tok] * invT - M - __logf(rs.Z);
  }
  }  // passes B, C, D
}

int sample_chunks(int B, int V, int wgs) {
  static const int forced = [] {
    const char* e = std::getenv("AKAP_SAMPLE_CHUNKS");
    return e ? std::atoi(e) : 0;
  }();
  const int need = (V + kMaxTiles * kTile - 1) / (kMaxTiles * kTile);  // <= kMaxTiles tiles
  if (forced > 0) return max(need, min(forced, kMaxChunks));
  // ~wgs workgroups over the batch (each chunk streams its share with 4 loads in flight per
  // thread; more, smaller chunks pay the per-workgroup publish / ticket / combine latency more
  // often: profiles/r5_sampler_rework_2.md), chunks of >= 2k elements, at most kMaxChunks
  int S = (wgs + B - 1) / max(B, 1);
  S = min(S, max(1, V / 2048));
  S = max(S, need);
  return max(1, min(S, kMaxChunks));
}

long sample_ws_floats(int B) {
  // partial records, selection states, per-row histograms (kMaxChunks x 512 float2), the
  // draw rows' tile masses (kMaxChunks x kMaxTiles)
  return (long)B * (kMaxChunks * 8 + kSelWords + 2 * kHistRow + kMaxChunks * kMaxTiles);
}

// Chunks per row of the filter passes: each pass has a fixed cost per workgroup (publish,
// ticket, two round trips), so they take fewer, larger chunks -- ~512 workgroups per pass
// over the batch (one round on 256 CUs), at most sample_chunks
static int filter_chunks(int B, int V) {
  return max(1, min(sample_chunks(B, V, 512), 512 / max(B, 1)));
}

void launch_sample(const SampleParams& p, int B, void* ws, int* tickets, int filtered,
                   hipStream_t s) {
  if (B == 0) return;
  // filtered batches: twice the chunks (the chunk kernel visits each chunk twice, and more
  // waves per SIMD hide its per-element work)
  const dim3 grid(sample_chunks(B, p.V, filtered ? 1024 : 512), B);
  const dim3 gridf(filter_chunks(B, p.V), B);
  SampPart* parts = (SampPart*)ws;
  SelState* st = reinterpret_cast<SelState*>(parts + (size_t)B * kMaxChunks);
  float2* hist = reinterpret_cast<float2*>(st + B);
  float* rowsum = reinterpret_cast<float*>(st);
  float* tiles = reinterpret_cast<float*>(hist + (size_t)B * kHistRow);
  if (p.is_bf16) {
    sample_chunk_kernel<bf16><<<grid, kChunkThreads, 0, s>>>(p, parts, tickets, rowsum, tiles,
                                                             hist);
    if (filtered) {
      sample_pass_kernel<bf16, true><<<gridf, kChunkThreads, 0, s>>>(p, 0, st, hist, tickets);
      for (int ps = 1; ps < 4; ++ps)
        sample_pass_kernel<bf16, false><<<gridf, kChunkThreads, 0, s>>>(p, ps, st, hist, tickets);
    }
  } else {
    sample_chunk_kernel<float><<<grid, kChunkThreads, 0, s>>>(p, parts, tickets, rowsum, tiles,
                                                             hist);
    if (filtered) {
      sample_pass_kernel<float, true><<<gridf, kChunkThreads, 0, s>>>(p, 0, st, hist, tickets);
      for (int ps = 1; ps < 4; ++ps)
        sample_pass_kernel<float, false><<<gridf, kChunkThreads, 0, s>>>(p, ps, st, hist, tickets);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void apply_penalties_kernel(
    T* __restrict__ logits, int ld, const int32_t* __restrict__ rows,
    const int32_t* __restrict__ toks, const int32_t* __restrict__ counts,
    const float* __restrict__ presence, const float* __restrict__ frequency,
    const float* __restrict__ repetition, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int r = rows[i];
  const int c = counts[i];
  T* px = logits + (size_t)r * ld + toks[i];
  float x = (float)*px;
  const float rep = repetition[r];
  if (rep != 1.f) x = x > 0.f ? x / rep : x * rep;
  x -= frequency[r] * (float)c + (c > 0 ? presence[r] : 0.f);
  *px = (T)x;
}

void launch_apply_penalties(void* logits, int ld, int is_bf16, const int32_t* rows,
                            const int32_t* toks, const int32_t* counts, const float* presence,
                            const float* frequency, const float* repetition, int n,
                            hipStream_t s) {
  if (n == 0) return;
  const int blocks = (n + 255) / 256;
  if (is_bf16)
    apply_penalties_kernel<bf16><<<blocks, 256, 0, s>>>((bf16*)logits, ld, rows, toks, counts,
                                                       presence, frequency, repetition, n);
  else
    apply_penalties_kernel<float><<<blocks, 256, 0, s>>>((float*)logits, ld, rows, toks, counts,
                                                        presence, frequency, repetition, n);
}

// Greedy fast path straight on bf16 or fp32 logits.
template <typename T>
__global__ __launch_bounds__(1024) void argmax_kernel(const T* logits, int ld, int V,
                                                      int64_t* out) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const int row = blockIdx.x;
  const T* x = logits + (size_t)row * ld;
  ArgBest b{-INFINITY, 0x7fffffff};
  // 8 contiguous elements per thread per step (16 B for bf16)
  const int nvec = V / 8;
  for (int v = threadIdx.x; v < nvec; v += blockDim.x) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = (float)x[v * 8 + j];
      if (f > b.v) { b.v = f; b.i = v * 8 + j; }
    }
  }
  for (int i = nvec * 8 + threadIdx.x; i < V; i += blockDim.x) {
    const float f = (float)x[i];
    if (f > b.v) { b.v = f; b.i = i; }
  }
  b = block_argmax(b, sv, si);
  if (threadIdx.x == 0) out[row] = b.i;
}

void launch_argmax(const void* logits, int ld, int V, int is_bf16, int64_t* out, int B,
                   hipStream_t s) {
  if (B == 0) return;
  if (is_bf16)
    argmax_kernel<bf16><<<B, 1024, 0, s>>>((const bf16*)logits, ld, V, out);
  else
    argmax_kernel<float><<<B, 1024, 0, s>>>((const float*)logits, ld, V, out);
}

}  // namespace akap
