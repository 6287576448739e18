// RMSNorm and fused residual-add + RMSNorm for gfx950.
//
// Memory-bound: one wave per row, 16-byte (8 x bf16) vector loads, the whole
// row held in VGPRs between the reduction and the write (no second HBM read).
// Reduction is wave-local (__shfl_xor over 64 lanes) so there is no LDS and
// no barrier on the critical path.  4 rows per 256-thread workgroup.
#include "common.h"
#include "kernels.h"

namespace akap {

template <int NV, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_wave_kernel(
    bf16* __restrict__ out, bf16* __restrict__ residual, const bf16* __restrict__ x,
    const bf16* __restrict__ w, int rows, int d, int x_stride, int out_stride, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16* xr = x + (size_t)row * x_stride;
  bf16x8 v[NV];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 8;
    v[i] = *reinterpret_cast<const bf16x8*>(xr + c);
  }
  if constexpr (ADD) {
    bf16* rr = residual + (size_t)row * d;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 8;
      bf16x8 r = *reinterpret_cast<const bf16x8*>(rr + c);
      bf16x8 s;
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] = f2bf(bf2f(v[i][j]) + bf2f(r[j]));
      v[i] = s;
      *reinterpret_cast<bf16x8*>(rr + c) = s;
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = bf2f(v[i][j]);
      ss += f * f;
    }
  ss = wave_sum(ss);
  const float inv = rsqrtf(ss / (float)d + eps);
  bf16* orow = out + (size_t)row * out_stride;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 8;
    bf16x8 wv = *reinterpret_cast<const bf16x8*>(w + c);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(v[i][j]) * inv * bf2f(wv[j]));
    *reinterpret_cast<bf16x8*>(orow + c) = o;
  }
}

// Few long rows (decode: 256 x 4096 / 8192): one 256-thread workgroup per row, VPT 16-byte
// vectors per thread, every load (x, residual, weight) issued before the reduction; wave sums
// meet in LDS.  The one-wave-per-row kernel puts only rows/4 workgroups on the chip (64 CUs at
// 256 rows) and serialises 8-16 dependent vector loads per lane.
template <int VPT, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_row_kernel(
    bf16* __restrict__ out, bf16* __restrict__ residual, const bf16* __restrict__ x,
    const bf16* __restrict__ w, int rows, int d, int x_stride, int out_stride, float eps) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const bf16* xr = x + (size_t)row * x_stride;
  bf16x8 v[VPT], wv[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (i * 256 + threadIdx.x) * 8;
    v[i] = *reinterpret_cast<const bf16x8*>(xr + c);
    wv[i] = *reinterpret_cast<const bf16x8*>(w + c);
  }
  if constexpr (ADD) {
    bf16* rr = residual + (size_t)row * d;
    bf16x8 r[VPT];
#pragma unroll
    for (int i = 0; i < VPT; ++i) r[i] = *reinterpret_cast<const bf16x8*>(rr + (i * 256 + threadIdx.x) * 8);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      bf16x8 s;
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] = f2bf(bf2f(v[i][j]) + bf2f(r[i][j]));
      v[i] = s;
      *reinterpret_cast<bf16x8*>(rr + (i * 256 + threadIdx.x) * 8) = s;
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = bf2f(v[i][j]);
      ss += f * f;
    }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / (float)d + eps);
  bf16* orow = out + (size_t)row * out_stride;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(v[i][j]) * inv * bf2f(wv[i][j]));
    *reinterpret_cast<bf16x8*>(orow + (i * 256 + threadIdx.x) * 8) = o;
  }
}

// Generic fallback: any d that is a multiple of 8, one workgroup per row.
template <bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_generic_kernel(
    bf16* __restrict__ out, bf16* __restrict__ residual, const bf16* __restrict__ x,
    const bf16* __restrict__ w, int rows, int d, int x_stride, int out_stride, float eps) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const bf16* xr = x + (size_t)row * x_stride;
  bf16* rr = ADD ? residual + (size_t)row * d : nullptr;
  float ss = 0.f;
  for (int c = threadIdx.x * 8; c < d; c += blockDim.x * 8) {
    bf16x8 v = *reinterpret_cast<const bf16x8*>(xr + c);
    if constexpr (ADD) {
      bf16x8 r = *reinterpret_cast<const bf16x8*>(rr + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = f2bf(bf2f(v[j]) + bf2f(r[j]));
      *reinterpret_cast<bf16x8*>(rr + c) = v;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += bf2f(v[j]) * bf2f(v[j]);
  }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / (float)d + eps);
  bf16* orow = out + (size_t)row * out_stride;
  const bf16* src = ADD ? rr : xr;
  for (int c = threadIdx.x * 8; c < d; c += blockDim.x * 8) {
    bf16x8 v = *reinterpret_cast<const bf16x8*>(src + c);
    bf16x8 wv = *reinterpret_cast<const bf16x8*>(w + c);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(v[j]) * inv * bf2f(wv[j]));
    *reinterpret_cast<bf16x8*>(orow + c) = o;
  }
}

template <bool ADD>
static void dispatch_rmsnorm(void* out, void* residual, const void* x, const void* w, int rows,
                             int d, int x_stride, int out_stride, float eps, hipStream_t s) {
  if (rows == 0) return;
  auto o = (bf16*)out;
  auto r = (bf16*)residual;
  auto xi = (const bf16*)x;
  auto wi = (const bf16*)w;
  dim3 grid((rows + 3) / 4), block(256);
  if (rows <= 1024 && d % 2048 == 0 && d <= 8192) {
    switch (d / 2048) {
#define RCASE(N)                                                                            \
  case N:                                                                                   \
    rmsnorm_row_kernel<N, ADD><<<rows, 256, 0, s>>>(o, r, xi, wi, rows, d, x_stride,       \
                                                    out_stride, eps);                       \
    return;
      RCASE(1) RCASE(2) RCASE(3) RCASE(4)
#undef RCASE
      default: break;
    }
  }
  if (d % 512 == 0 && d <= 8192) {
    switch (d / 512) {
#define CASE(N)                                                                             \
  case N:                                                                                   \
    rmsnorm_wave_kernel<N, ADD><<<grid, block, 0, s>>>(o, r, xi, wi, rows, d, x_stride,    \
                                                       out_stride, eps);                   \
    return;
      CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
      CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
      default: break;
    }
  }
  rmsnorm_generic_kernel<ADD><<<rows, 256, 0, s>>>(o, r, xi, wi, rows, d, x_stride, out_stride,
                                                   eps);
}

void launch_rmsnorm(void* out, const void* x, const void* w, int rows, int d, int x_stride,
                    int out_stride, float eps, hipStream_t s) {
  dispatch_rmsnorm<false>(out, nullptr, x, w, rows, d, x_stride, out_stride, eps, s);
}

void launch_fused_add_rmsnorm(void* out, void* residual, const void* x, const void* w, int rows,
                              int d, int x_stride, int out_stride, float eps, hipStream_t s) {
  dispatch_rmsnorm<true>(out, residual, x, w, rows, d, x_stride, out_stride, eps, s);
}

}  // namespace akap
