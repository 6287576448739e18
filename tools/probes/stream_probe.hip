// HBM streaming-read rate on one MI355X by load path, to size what the decode attention (the
// KV stream, 69 % of the Qwen3 decode step) could gain from its load path alone:
//   reg     global_load_dwordx4 into VGPRs, 8 loads in flight per lane (the attention's path)
//   lds     global_load_lds_dwordx4 (LDS-DMA) into a 4-slot ring per wave, counted vmcnt
//   lds_nt  the same with the non-temporal cache policy
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/stream_probe tools/probes/stream_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_reg(const u32x4* __restrict__ p, size_t n, unsigned* out) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  for (; i + 7 * stride < n; i += 8 * stride) {
    u32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = __builtin_nontemporal_load(p + i + j * stride);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc ^= v[j];
  }
  for (; i < n; i += stride) acc ^= p[i];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

template <int AUX>
__global__ __launch_bounds__(256) void k_lds(const u32x4* __restrict__ p, size_t n, unsigned* out) {
  // each wave streams its own 1 KiB pieces through an 8-slot x 1 KiB ring: 7 pieces in flight,
  // counted waits (never vmcnt(0) in the steady state)
  __shared__ u32x4 ring[4][8][64];  // [wave][slot][lane]
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t waves = (size_t)gridDim.x * 4;
  const size_t wid = (size_t)blockIdx.x * 4 + w;
  const size_t pieces = n / 64;  // 1 KiB pieces
  const size_t mine = pieces > wid ? (pieces - wid + waves - 1) / waves : 0;
  auto issue = [&](size_t q) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(p + (wid + q * waves) * 64 + lane),
        (__attribute__((address_space(3))) void*)&ring[w][q & 7][0], 16, 0, AUX);
  };
  unsigned acc = 0;
  if (mine < 8) {
    for (size_t q = 0; q < mine; ++q) issue(q);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (size_t q = 0; q < mine; ++q) acc ^= ring[w][q & 7][lane].x;
  } else {
    for (size_t q = 0; q < 7; ++q) issue(q);
    for (size_t q = 0; q < mine; ++q) {
      if (q + 7 < mine) {
        issue(q + 7);
        asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      acc ^= ring[w][q & 7][lane].x;
    }
  }
  if (acc == 0x12345678u) out[0] = 1;
}

template <typename F>
static double timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const size_t bytes = (size_t)8 << 30;
  const size_t n = bytes / 16;
  u32x4* p;
  unsigned* out;
  CK(hipMalloc(&p, bytes));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(p, 1, bytes));
  for (int grid : {1024, 2048, 4096}) {
    double t = timeit([&] { k_reg<<<grid, 256>>>(p, n, out); }, 5);
    printf("reg     grid %5d: %.2f TB/s\n", grid, bytes / t / 1e9);
    t = timeit([&] { k_lds<0><<<grid, 256>>>(p, n, out); }, 5);
    printf("lds     grid %5d: %.2f TB/s\n", grid, bytes / t / 1e9);
    t = timeit([&] { k_lds<2><<<grid, 256>>>(p, n, out); }, 5);
    printf("lds_nt  grid %5d: %.2f TB/s\n", grid, bytes / t / 1e9);
    fflush(stdout);
  }
  CK(hipGetLastError());
  CK(hipFree(p));
  return 0;
}
