// Token sampling for gfx950: greedy, temperature, top-k, top-p in one launch.
//
// No sort: top-k / top-p thresholds are found by a radix select on the order-preserving
// uint32 image of the logits -- by COUNT for top-k and by probability MASS for top-p.  The
// draw is a Gumbel-max over the surviving set with a counter-based RNG keyed by (request
// seed, request step, token id), so a request's stream is reproducible regardless of batch
// composition.  The row is split over several workgroups (sample_chunk_kernel below).
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
// Two launches.  A row of V ~ 152k logits is ~300 KB: one workgroup per row leaves most of
// the 256 CUs idle at decode batch sizes (B = 64 -> 64 CUs) and re-streams the row per pass.
//
// 1. sample_chunk_kernel, grid = (S chunks, B rows): every workgroup reads its chunk ONCE
//    with 16-byte vector loads and produces, in that single pass,
//      greedy rows   the chunk's argmax (first index on ties);
//      T > 0 rows    the chunk's max and partition sum of z = x / T (online: rescaled when the
//                    max moves) and, for rows with top-k / top-p, the key range.
//    The chunk publishes a 32-byte partial record with write-through (sc1) stores and takes
//    a ticket on the row's counter (MI355X_MICROARCH.md "Valid forms", sc1 table row 1: no
//    release / acquire fence -- each costs ~1.7 us and more behind a freshly written logits
//    tensor); the LAST chunk of the row reads the S records with sc1 loads, combines them
//    (max, rescaled sum), re-arms the counter and writes the token + log-prob of a greedy row,
//    or the row summary (M, Z, key range) of a row with filters; a row without filters is
//    drawn there by inverse CDF: u(seed, step) * Z picks the chunk from the prefix of the
//    chunk masses, then the workgroup rescans that one chunk (a block scan of per-thread run
//    masses) for the token -- exact sampling with one exp per element in the main pass and
//    no per-element RNG.
// 2. sample_filter_kernel, grid = B: rows with top-k / top-p (the others return at once) find
//    their thresholds by an adaptive radix select over the order-preserving key image -- by
//    COUNT for top-k, by probability MASS for top-p on the top-k renormalised distribution:
//    256 bins over the row's live key interval, the bin width a power of two, so bf16 logits
//    (16-bit keys) take exactly 2 passes; per-lane copies of the histogram (bin-major, so a
//    wave's 64 lanes always hit 64 different banks and never the same word) -- then the
//    Gumbel draw over the survivors.
constexpr int kChunkThreads = 256;
constexpr int kMaxChunks = 64;
constexpr int kFilterThreads = 256;
constexpr int kSc1 = 16;  // buffer op cache bits: sc1 (write-through stores, L1-bypass loads)

struct SampPart {  // one chunk's partial record (32 B = two 16-B vectors)
  float m, s;      // max of z over the chunk, sum of exp(z - m)
  float unused0;
  int unused1;
  float am;        // argmax value (greedy rows)
  int ai;
  uint32_t kmin, kmax;  // key range of the chunk
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

// Visit x[lo, hi) as (value, index) with 16-byte loads where the row is aligned.
template <typename T, typename F>
__device__ __forceinline__ void visit_range(const T* x, int lo, int hi, bool vec_ok, F&& f) {
  constexpr int NV = Vec<T>::N;
  if (vec_ok) {
    const int vlo = (lo + NV - 1) / NV, vhi = hi / NV;
    for (int i = lo + threadIdx.x; i < min(hi, vlo * NV); i += blockDim.x) f((float)x[i], i);
    for (int v = vlo + threadIdx.x; v < vhi; v += blockDim.x) {
      const typename Vec<T>::type q =
          *reinterpret_cast<const typename Vec<T>::type*>(x + (size_t)v * NV);
#pragma unroll
      for (int j = 0; j < NV; ++j) f((float)q[j], v * NV + j);
    }
    for (int i = max(vhi * NV, vlo * NV) + threadIdx.x; i < hi; i += blockDim.x) f((float)x[i], i);
  } else {
    for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) f((float)x[i], i);
  }
}

__device__ __forceinline__ bool row_filtered(const SampleParams& p, int row, float temp) {
  if (!(temp > 0.f)) return false;
  const int k = p.top_k ? p.top_k[row] : 0;
  const float tp = p.top_p ? p.top_p[row] : 1.f;
  return (k > 0 && k < p.V) || (tp < 1.f && tp > 0.f);
}

template <typename T>
__global__ __launch_bounds__(kChunkThreads) void sample_chunk_kernel(SampleParams p, SampPart* ws,
                                                                     int* tickets, float* rowsum) {
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
  uint32_t kmin = 0xffffffffu, kmax = 0u;
  ArgBest best{-INFINITY, 0x7fffffff};
  if (!need_sum) {
    visit_range(x, lo, hi, vec_ok, [&](float v, int i) {
      if (v > best.v) { best.v = v; best.i = i; }  // ascending i per thread: first max kept
    });
  } else if (!greedy && !filt) {
    // max and partition sum only (one exp per element): the draw is an inverse-CDF pick by
    // the last chunk below, so no per-element RNG / logs in this pass
    visit_range(x, lo, hi, vec_ok, [&](float v, int) {
      const float z = v * invT;
      if (z > m) { sum = sum * __expf(m - z) + 1.f; m = z; }
      else if (z > -INFINITY) sum += __expf(z - m);
    });
  } else {  // greedy with log-probs, or a filtered row (also its key range)
    visit_range(x, lo, hi, vec_ok, [&](float v, int i) {
      if (v > best.v) { best.v = v; best.i = i; }
      const float z = v * invT;
      if (z > m) { sum = sum * __expf(m - z) + 1.f; m = z; }
      else if (z > -INFINITY) sum += __expf(z - m);
      const uint32_t k = fkey(v);
      kmin = min(kmin, k);
      kmax = max(kmax, k);
    });
  }
  // workgroup reductions
  if (!need_sum || greedy) best = block_argmax(best, sv, si);
  float M = -INFINITY, Z = 0.f;
  if (need_sum) {
    M = block_max(m, sv);
    Z = block_sum(m == -INFINITY ? 0.f : sum * __expf(m - M), sv);
  }
  __shared__ uint32_t s_kmin, s_kmax;
  if (filt) {  // exact integer min / max of the keys
    if (threadIdx.x == 0) { s_kmin = 0xffffffffu; s_kmax = 0u; }
    __syncthreads();
    atomicMin(&s_kmin, kmin);
    atomicMax(&s_kmax, kmax);
    __syncthreads();
    kmin = s_kmin;
    kmax = s_kmax;
  }
  // ---- publish the partial (sc1 stores), take a ticket ----
  const __amdgpu_buffer_rsrc_t rws = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(ws + (size_t)row * S), (short)0, (int)(S * sizeof(SampPart)), 0x00020000);
  if (threadIdx.x == 0) {
    u32x4 a, b2;
    a[0] = __float_as_uint(M); a[1] = __float_as_uint(Z);
    a[2] = 0u; a[3] = 0u;
    b2[0] = __float_as_uint(best.v); b2[1] = (uint32_t)best.i; b2[2] = kmin; b2[3] = kmax;
    __builtin_amdgcn_raw_buffer_store_b128(a, rws, c * 32, 0, kSc1);
    __builtin_amdgcn_raw_buffer_store_b128(b2, rws, c * 32 + 16, 0, kSc1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int t = __hip_atomic_fetch_add(tickets + row * kCtrStride, 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == S - 1;
  }
  __syncthreads();
  if (!s_last) return;
  // ---- last chunk of the row: combine the S partials (S <= 64: wave 0, sc1 loads) ----
  const bool draw = !greedy && !filt;  // uniform over the workgroup
  __shared__ float s_m, s_z, s_res;
  __shared__ int s_chunk, s_tok, s_fb;
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    float rm = -INFINITY, rs = 0.f;
    ArgBest a{-INFINITY, 0x7fffffff};
    uint32_t rkmin = 0xffffffffu, rkmax = 0u;
    if (l < S) {
      const u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(rws, l * 32, 0, kSc1);
      const u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(rws, l * 32 + 16, 0, kSc1);
      rm = __uint_as_float(v0[0]); rs = __uint_as_float(v0[1]);
      a = ArgBest{__uint_as_float(v1[0]), (int)v1[1]};
      rkmin = v1[2]; rkmax = v1[3];
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
      rkmin = min(rkmin, (uint32_t)__shfl_xor((int)rkmin, o, 64));
      rkmax = max(rkmax, (uint32_t)__shfl_xor((int)rkmax, o, 64));
    }
    if (draw) {
      // inverse CDF, level 1: the chunk whose prefix mass first reaches u * Z
      const float target = uniform01(seed, step, 0xffffffffu) * Zr;
      const uint64_t hit = __ballot(incl >= target && w > 0.f);
      const uint64_t live = __ballot(w > 0.f);
      const int c_sel = hit ? __builtin_ctzll(hit) : 63 - __builtin_clzll(live);
      if (l == c_sel) {
        s_chunk = l;
        s_res = hit ? target - (incl - w) : w;  // rounding past the end: the chunk's last mass
      }
      if (l == 0) {
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
      } else if (filt) {  // sample_filter_kernel finishes the row
        float* r = rowsum + (size_t)row * 4;
        r[0] = Mr;
        r[1] = Zr;
        r[2] = __uint_as_float(rkmin);
        r[3] = __uint_as_float(rkmax);
      }
    }
  }
  if (!draw) return;
  __syncthreads();
  // ---- inverse CDF, level 2: rescan the selected chunk (just read by its workgroup, so in
  // L2), each thread a contiguous run; block exclusive scan of the run masses; the thread
  // whose run crosses the residual mass walks it to the token ----
  const float Mr = s_m, R = s_res;
  const int lo2 = min(V, s_chunk * chunk), hi2 = min(V, lo2 + chunk);
  const int per = (hi2 - lo2 + kChunkThreads - 1) / kChunkThreads;
  const int a0 = min(hi2, lo2 + (int)threadIdx.x * per), a1 = min(hi2, a0 + per);
  float ts = 0.f;
  int last_pos = -1;
  for (int i = a0; i < a1; ++i) {
    const float e = __expf((float)x[i] * invT - Mr);
    ts += e;
    if (e > 0.f) last_pos = i;
  }
  // exclusive scan of ts over the workgroup (waves scan, then the 4 wave totals)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float inc = ts;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) sv[wid] = inc;
  __syncthreads();
  float before = inc - ts;
  for (int wv = 0; wv < wid; ++wv) before += sv[wv];
  if (last_pos >= 0) atomicMax(&s_fb, last_pos);
  if (ts > 0.f && R >= before && R < before + ts) {
    float acc = before;
    int tok = last_pos;
    for (int i = a0; i < a1; ++i) {
      acc += __expf((float)x[i] * invT - Mr);
      if (acc > R) { tok = i; break; }
    }
    atomicMin(&s_tok, tok);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int tok = s_tok != 0x7fffffff ? s_tok : s_fb;  // rounding past the chunk's end: last mass
    if (tok < 0 || tok >= V) tok = 0;
    p.out_tokens[row] = tok;
    if (p.out_logprobs) p.out_logprobs[row] = (float)x[tok] * invT - Mr - __logf(s_z);
  }
}

// Largest key tau in [floor_key, kmax] with sum_{key >= tau} w >= target, w = 1 (MASS=false)
// or exp(x/T - M) (MASS=true); returns floor_key when the whole interval holds less.
template <bool MASS, typename T>
__device__ uint32_t adaptive_select(const T* x, int V, bool vec_ok, uint32_t floor_key,
                                    uint32_t kmax, float target, float M, float invT,
                                    float* hist /* [256][64] */, uint32_t* s_u, float* s_f) {
  const int tid = threadIdx.x, lane = tid & 63;
  uint32_t lo = floor_key, hi = kmax;
  float remaining = target;
  while (hi > lo) {
    const uint64_t range = (uint64_t)hi - lo + 1;
    int sh = 0;
    while ((range + ((1ull << sh) - 1)) >> sh > 256) ++sh;  // bins of width 2^sh, <= 256 bins
    for (int i = tid; i < 256 * 64; i += blockDim.x) hist[i] = 0.f;
    __syncthreads();
    const uint32_t lo_ = lo, hi_ = hi;
    visit_range(x, 0, V, vec_ok, [&](float v, int) {
      const uint32_t k = fkey(v);
      if (k < lo_ || k > hi_) return;
      const int b = (int)((k - lo_) >> sh);
      atomicAdd(&hist[b * 64 + lane], MASS ? __expf(v * invT - M) : 1.f);
    });
    __syncthreads();
    // per-bin totals over the 64 copies (rotated reads: conflict-free), then one wave scans
    float* tot = hist;  // reused in place below after a barrier
    float bsum = 0.f;
    {
      const int b = tid;  // blockDim == 256 bins
#pragma unroll 8
      for (int j = 0; j < 64; ++j) bsum += hist[b * 64 + ((j + lane) & 63)];
    }
    __syncthreads();
    tot[tid] = bsum;
    __syncthreads();
    if (tid < 64) {
      float c[4], loc = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c[j] = tot[255 - 4 * lane - j];
        loc += c[j];
      }
      float incl = loc;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
      }
      const float before = incl - loc;
      const uint64_t ball = __ballot(before + loc >= remaining);
      const int first = ball ? __builtin_ctzll(ball) : 64;
      if (first == 64) {  // the interval holds less than the target: take all of it
        if (lane == 0) { s_u[0] = 0xffffffffu; s_f[0] = remaining; }
      } else if (lane == first) {
        float cum = before;
        int sel = 252 - 4 * lane;
        for (int j = 0; j < 4; ++j) {
          sel = 255 - 4 * lane - j;
          if (cum + c[j] >= remaining) break;
          cum += c[j];
        }
        s_u[0] = (uint32_t)sel;
        s_f[0] = remaining - cum;
      }
    }
    __syncthreads();
    const uint32_t sel = s_u[0];
    remaining = s_f[0];
    __syncthreads();
    if (sel == 0xffffffffu) return lo;
    lo = lo + (sel << sh);
    const uint64_t top = (uint64_t)lo + (1ull << sh) - 1;
    hi = top < hi ? (uint32_t)top : hi;
  }
  return lo;
}

template <typename T>
__global__ __launch_bounds__(kFilterThreads) void sample_filter_kernel(SampleParams p,
                                                                       const float* rowsum) {
  __shared__ float hist[256 * 64];
  __shared__ float sv[16];
  __shared__ int si[16];
  __shared__ uint32_t s_u[1];
  __shared__ float s_f[1];
  const int row = blockIdx.x;
  const float temp = p.temperature ? p.temperature[row] : 0.f;
  if (!row_filtered(p, row, temp)) return;  // uniform: the whole workgroup leaves
  const T* x = reinterpret_cast<const T*>(p.logits) + (size_t)row * p.ld;
  const int V = p.V;
  const bool vec_ok = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  const float invT = 1.f / temp;
  const float M = rowsum[row * 4], Z = rowsum[row * 4 + 1];
  const uint32_t kmin = __float_as_uint(rowsum[row * 4 + 2]);
  const uint32_t kmax = __float_as_uint(rowsum[row * 4 + 3]);
  const int k = p.top_k ? p.top_k[row] : 0;
  const float tp = p.top_p ? p.top_p[row] : 1.f;
  uint32_t thr = kmin;
  float Zk = Z;
  if (k > 0 && k < V) {
    thr = adaptive_select<false>(x, V, vec_ok, kmin, kmax, (float)k, M, invT, hist, s_u, s_f);
    if (tp < 1.f) {
      float zk = 0.f;
      visit_range(x, 0, V, vec_ok, [&](float v, int) {
        if (fkey(v) >= thr) zk += __expf(v * invT - M);
      });
      Zk = block_sum(zk, sv);
    }
  }
  if (tp < 1.f && tp > 0.f)
    thr = adaptive_select<true>(x, V, vec_ok, thr, kmax, tp * Zk, M, invT, hist, s_u, s_f);
  // Gumbel-max draw over {key >= thr}
  const uint64_t seed = p.seeds ? (uint64_t)p.seeds[row] : 0x1234ull + row;
  const uint32_t step = p.steps ? (uint32_t)p.steps[row] : 0u;
  ArgBest b{-INFINITY, 0x7fffffff};
  visit_range(x, 0, V, vec_ok, [&](float v, int i) {
    if (fkey(v) < thr) return;
    const float u = uniform01(seed, step, (uint32_t)i);
    const float g = v * invT - __logf(-__logf(u));
    if (g > b.v) { b.v = g; b.i = i; }
  });
  b = block_argmax(b, sv, si);
  if (threadIdx.x == 0) {
    int tok = b.i;
    if (tok < 0 || tok >= V) tok = 0;
    p.out_tokens[row] = tok;
    if (p.out_logprobs) p.out_logprobs[row] = (float)x[tok] * invT - M - __logf(Z);
  }
}

int sample_chunks(int B, int V) {
  // ~2k workgroups over the batch, chunks of >= 2k elements, at most kMaxChunks per row
  int S = (2048 + B - 1) / max(B, 1);
  S = min(S, max(1, V / 2048));
  return max(1, min(S, kMaxChunks));
}

void launch_sample(const SampleParams& p, int B, void* ws, int* tickets, hipStream_t s) {
  if (B == 0) return;
  const dim3 grid(sample_chunks(B, p.V), B);
  // workspace: [B][kMaxChunks] partial records, then [B][4] row summaries
  SampPart* parts = (SampPart*)ws;
  float* rowsum = reinterpret_cast<float*>(parts + (size_t)B * kMaxChunks);
  if (p.is_bf16) {
    sample_chunk_kernel<bf16><<<grid, kChunkThreads, 0, s>>>(p, parts, tickets, rowsum);
    sample_filter_kernel<bf16><<<B, kFilterThreads, 0, s>>>(p, rowsum);
  } else {
    sample_chunk_kernel<float><<<grid, kChunkThreads, 0, s>>>(p, parts, tickets, rowsum);
    sample_filter_kernel<float><<<B, kFilterThreads, 0, s>>>(p, rowsum);
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
