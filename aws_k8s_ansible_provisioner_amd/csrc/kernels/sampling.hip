// Token sampling for gfx950: greedy, temperature, top-k, top-p in one kernel.
//
// One 1024-thread workgroup per row (vocab up to ~256k; the row stays L2-resident
// across passes).  No sort: top-k / top-p thresholds are found by a 4-pass 8-bit
// radix select on the order-preserving uint32 image of the logits -- by COUNT for
// top-k and by probability MASS for top-p -- with LDS histograms.  The draw is a
// Gumbel-max over the surviving set with a counter-based RNG keyed by
// (request seed, request step, token id), so a request's stream is reproducible
// regardless of batch composition.
#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int kSampThreads = 1024;

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

template <typename T>
__device__ __forceinline__ float ldf(const T* p, int i) { return (float)p[i]; }

template <typename T>
__device__ ArgBest row_argmax(const T* x, int V, float* sv, int* si) {
  ArgBest b{-INFINITY, 0x7fffffff};
  int tail = 0;
  if constexpr (sizeof(T) == 2) {
    // 16-byte vector loads: 8 contiguous bf16 per lane per step
    if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
      const int nvec = V / 8;
      for (int v = threadIdx.x; v < nvec; v += blockDim.x) {
        const bf16x8 q = *reinterpret_cast<const bf16x8*>(x + (size_t)v * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = (float)q[j];
          if (f > b.v) { b.v = f; b.i = v * 8 + j; }
        }
      }
      tail = nvec * 8;
    }
  }
  for (int i = tail + threadIdx.x; i < V; i += blockDim.x) {
    const float v = ldf(x, i);
    if (v > b.v) { b.v = v; b.i = i; }  // strided ascending i: first max kept
  }
  return block_argmax(b, sv, si);
}

// Radix select over keys of x (restricted to key >= floor_key).
//  MASS=false: returns the key of the k-th largest element (k = target, integer).
//  MASS=true : returns the largest key tau with sum_{key>=tau} exp((x-M)*invT) >= target.
template <bool MASS, typename T>
__device__ uint32_t radix_select(const T* x, int V, uint32_t floor_key, float target,
                                 float M, float invT, int* cnt, float* mass, uint32_t* shared_u,
                                 float* shared_f) {
  uint32_t prefix = 0, mask = 0;
  float remaining = target;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int b = threadIdx.x; b < 256; b += blockDim.x) { cnt[b] = 0; mass[b] = 0.f; }
    __syncthreads();
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      const float v = (float)x[i];
      const uint32_t k = fkey(v);
      if (k < floor_key || (k & mask) != prefix) continue;
      const int d = (k >> shift) & 255;
      if (MASS)
        atomicAdd(&mass[d], __expf((v - M) * invT));
      else
        atomicAdd(&cnt[d], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float cum = 0.f;
      int sel = 0;
      for (int b = 255; b >= 0; --b) {
        const float c = MASS ? mass[b] : (float)cnt[b];
        if (cum + c >= remaining) { sel = b; remaining -= cum; break; }
        cum += c;
        if (b == 0) { sel = 0; remaining -= cum - c; }
      }
      shared_u[0] = (uint32_t)sel;
      shared_f[0] = remaining;
    }
    __syncthreads();
    prefix |= shared_u[0] << shift;
    mask |= 255u << shift;
    remaining = shared_f[0];
    __syncthreads();
  }
  return prefix;
}

template <typename T>
__global__ __launch_bounds__(kSampThreads) void sample_kernel(SampleParams p) {
  __shared__ float sv[16];
  __shared__ int si[16];
  __shared__ int cnt[256];
  __shared__ float mass[256];
  __shared__ uint32_t su[1];
  __shared__ float sf[1];
  const int row = blockIdx.x;
  const T* x = reinterpret_cast<const T*>(p.logits) + (size_t)row * p.ld;
  const int V = p.V;
  const float temp = p.temperature ? p.temperature[row] : 0.f;
  if (!(temp > 0.f)) {
    ArgBest b = row_argmax(x, V, sv, si);
    float lp = 0.f;
    if (p.greedy_logprobs && p.out_logprobs) {  // log-softmax of the argmax: -log sum exp(x-M)
      float z = 0.f;
      for (int i = threadIdx.x; i < V; i += blockDim.x) z += __expf((float)x[i] - b.v);
      lp = -__logf(block_sum(z, sv));
    }
    if (threadIdx.x == 0) {
      p.out_tokens[row] = b.i;
      if (p.out_logprobs) p.out_logprobs[row] = lp;
    }
    return;
  }
  const float invT = 1.f / temp;
  // pass 1: max and partition function
  float m = -INFINITY;
  for (int i = threadIdx.x; i < V; i += blockDim.x) m = fmaxf(m, (float)x[i]);
  const float M = block_max(m, sv);
  float z = 0.f;
  for (int i = threadIdx.x; i < V; i += blockDim.x) z += __expf(((float)x[i] - M) * invT);
  const float Z = block_sum(z, sv);

  uint32_t thr = 0;
  const int k = p.top_k ? p.top_k[row] : 0;
  const float tp = p.top_p ? p.top_p[row] : 1.f;
  float Zk = Z;
  if (k > 0 && k < V) {
    thr = radix_select<false>(x, V, 0, (float)k, M, invT, cnt, mass, su, sf);
    if (tp < 1.f) {
      float zk = 0.f;
      for (int i = threadIdx.x; i < V; i += blockDim.x)
        if (fkey((float)x[i]) >= thr) zk += __expf(((float)x[i] - M) * invT);
      Zk = block_sum(zk, sv);
    }
  }
  if (tp < 1.f && tp > 0.f) {
    const uint32_t t2 = radix_select<true>(x, V, thr, tp * Zk, M, invT, cnt, mass, su, sf);
    thr = t2 > thr ? t2 : thr;
  }
  // Gumbel-max draw over {key >= thr}
  const uint64_t seed = p.seeds ? (uint64_t)p.seeds[row] : 0x1234ull + row;
  const uint32_t step = p.steps ? (uint32_t)p.steps[row] : 0u;
  ArgBest b{-INFINITY, 0x7fffffff};
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float v = (float)x[i];
    if (fkey(v) < thr) continue;
    const float u = uniform01(seed, step, (uint32_t)i);
    const float gval = v * invT - __logf(-__logf(u));
    if (gval > b.v) { b.v = gval; b.i = i; }
  }
  b = block_argmax(b, sv, si);
  if (threadIdx.x == 0) {
    int tok = b.i;
    if (tok < 0 || tok >= V) tok = 0;
    p.out_tokens[row] = tok;
    if (p.out_logprobs) p.out_logprobs[row] = ((float)x[tok] - M) * invT - __logf(Z);
  }
}

void launch_sample(const SampleParams& p, int B, hipStream_t s) {
  if (B == 0) return;
  if (p.is_bf16)
    sample_kernel<bf16><<<B, kSampThreads, 0, s>>>(p);
  else
    sample_kernel<float><<<B, kSampThreads, 0, s>>>(p);
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
