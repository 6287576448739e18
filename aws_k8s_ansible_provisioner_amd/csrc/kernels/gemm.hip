// Decode-shape GEMM for gfx950:  Y[M,N] = X[M,K] . W[N,K]^T   (bf16 in, fp32 acc)
//
// The decode step's projections are M = batch (<= 512) against large weights: far from
// compute-bound, latency/L2-bound (cdna_hip_programming.md §5 "Projection GEMM at M=256").
// Library GEMMs pick tall tiles that leave most CUs idle (e.g. 128 WGs for N=4096), so
// this kernel uses small 64x64 output tiles + split-K to put >= 256 workgroups on the
// chip, XCD-aware tile order (tiles sharing a weight panel share an L2), and both
// operands K-major exactly as torch stores them (no transposes):
//   * MFMA v_mfma_f32_16x16x32_bf16: A = X rows, B = W rows (both 16-byte K-runs/lane);
//   * 4 waves as 2x2, each a 32x32 sub-tile = 2x2 MFMA tiles, BK = 64;
//   * global -> registers -> LDS double buffer (next tile's loads in flight during the
//     current tile's MFMAs), XOR-swizzled 16-byte chunks (conflict-free ds_read_b128);
//   * split-K partials go to an fp32 workspace [S, M, N] summed by a reduce pass
//     (or consumed directly by the fused residual-add + RMSNorm kernel).
#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int GBM = 64, GBN = 64, GBK = 64;

// LDS tile [64 rows][64 k] bf16 = 8 chunks of 16 B per row; chunk' = chunk ^ (row & 7).
__device__ __forceinline__ int swz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }

template <bool SPLIT, bool CHECK, bool INREDUCE = false>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(const bf16* __restrict__ X,
                                                        const bf16* __restrict__ W,
                                                        bf16* __restrict__ Y,
                                                        float* __restrict__ ws, int M, int N,
                                                        int K, int ldx, int ldw, int ldy,
                                                        int k_per_split,
                                                        int* __restrict__ counters) {
  // [buf][A|B][row*8+chunk]; the last element doubles as the split-K "last arriver" flag
  // (one __shared__ object: a second one makes hipcc drain vmcnt in the k-loop)
  __shared__ bf16x8 lds[2][2][GBM * 8];
  const int tiles_n = (N + GBN - 1) / GBN;
  const int tiles_m = (M + GBM - 1) / GBM;
  const int ntiles = tiles_n * tiles_m;
  // XCD-aware order: consecutive logical tiles (same weight panel, all M tiles) share an XCD
  const int lt = xcd_remap(blockIdx.x, ntiles);
  const int tn = lt / tiles_m;
  const int tm = lt % tiles_m;
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int kz = blockIdx.y;
  const int kbeg = kz * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;

  // staging: each thread moves 2 chunks of A and 2 of B per k-tile
  const int s_row = tid >> 2;        // 0..63
  const int s_ch = (tid & 3) * 2;    // chunk pair 0,2,4,6
  const bool a_ok = (m0 + s_row) < M;
  const bool b_ok = (n0 + s_row) < N;
  const bf16* xa = X + (size_t)(a_ok ? m0 + s_row : 0) * ldx;
  const bf16* wb = W + (size_t)(b_ok ? n0 + s_row : 0) * ldw;
  bf16x8 ra[2], rb[2];
  const bf16x8 zero8 = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};

  auto gload = [&](int k0) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int kk = k0 + (s_ch + c) * 8;
      if (CHECK) {
        ra[c] = (a_ok && kk < kend) ? *reinterpret_cast<const bf16x8*>(xa + kk) : zero8;
        rb[c] = (b_ok && kk < kend) ? *reinterpret_cast<const bf16x8*>(wb + kk) : zero8;
      } else {
        ra[c] = *reinterpret_cast<const bf16x8*>(xa + kk);
        rb[c] = *reinterpret_cast<const bf16x8*>(wb + kk);
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      lds[buf][0][swz(s_row, s_ch + c)] = ra[c];
      lds[buf][1][swz(s_row, s_ch + c)] = rb[c];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + GBK - 1) / GBK;
  if (nk > 0) {
    gload(kbeg);
    sstore(0);
  }
  __syncthreads();
  const int fr = lane & 15, fg = lane >> 4;
  for (int it = 0; it < nk; ++it) {
    const int cur = it & 1;
    if (it + 1 < nk) gload(kbeg + (it + 1) * GBK);  // in flight during the MFMAs below
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {  // two 32-deep MFMA k-steps per 64-deep tile
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = lds[cur][0][swz(wm * 32 + i * 16 + fr, ks * 4 + fg)];
        bfr[i] = lds[cur][1][swz(wn * 32 + i * 16 + fr, ks * 4 + fg)];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (it + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }
  // epilogue: lane holds rows fg*4 + r, col fr of each 16x16 tile
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 32 + j * 16 + fr;
      if (col >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + i * 16 + fg * 4 + r;
        if (row >= M) continue;
        if (SPLIT)
          ws[((size_t)kz * M + row) * N + col] = acc[i][j][r];
        else
          Y[(size_t)row * ldy + col] = f2bf(acc[i][j][r]);
      }
    }
  if constexpr (SPLIT && INREDUCE) {
    // In-launch split-K combine (cdna_hip_programming.md §5 "Projection GEMM at M = 256"
    // item 2): publish this slice's slab with an agent-scope release, take a ticket; the
    // slice drawing the last ticket acquires and sums all slabs of the tile into Y, then
    // re-arms the counter for the next call (graph-replay safe).  No reduce launch.
    const int S = gridDim.y;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(&lds[1][1][GBM * 8 - 1]);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(&counters[lt * kCtrStride], 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      *flag = old == S - 1;
    }
    __syncthreads();
    if (*flag) {
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        counters[lt * kCtrStride] = 0;
      }
      __syncthreads();
      // 64x64 tile, 256 threads: each thread 4 rows x 4 consecutive columns
      const int cc = (tid & 15) * 4;
      const int rr = tid >> 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = m0 + rr + 16 * q;
        const int col = n0 + cc;
        if (row >= M || col >= N) continue;
        f32x4 acc4 = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int z = 0; z < S; ++z)
          acc4 += *reinterpret_cast<const f32x4*>(ws + ((size_t)z * M + row) * N + col);
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = f2bf(acc4[j]);
        *reinterpret_cast<bf16x4*>(Y + (size_t)row * ldy + col) = o;
      }
    }
  }
}

// sum S fp32 partial slabs [S, M, N] -> bf16 Y
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws,
                                                            bf16* __restrict__ Y, int S, int M,
                                                            int N, int ldy) {
  const long total = (long)M * N / 4;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long e = i * 4;
    f32x4 s = *reinterpret_cast<const f32x4*>(ws + e);
    for (int z = 1; z < S; ++z) s += *reinterpret_cast<const f32x4*>(ws + (size_t)z * M * N + e);
    // 32-bit row/col split when the slab fits (a 64-bit division is a long software sequence)
    int row, col;
    if (total < (1L << 29)) {
      row = (int)e / N;
      col = (int)e - row * N;
    } else {
      row = (int)(e / N);
      col = (int)(e % N);
    }
    bf16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = f2bf(s[j]);
    *reinterpret_cast<bf16x4*>(Y + (size_t)row * ldy + col) = o;
  }
}

int gemm_splitk_choice(int M, int N, int K) {
  const int tiles = ((M + GBM - 1) / GBM) * ((N + GBN - 1) / GBN);
  int s = 1;
  while (tiles * s < 256 && K / (s * 2) >= 256) s *= 2;
  return s;
}

void launch_gemm_bf16(const void* X, const void* W, void* Y, float* ws, int M, int N, int K,
                      int ldx, int ldw, int ldy, int splitk, hipStream_t st, int* counters) {
  if (M == 0 || N == 0) return;
  const int tiles = ((M + GBM - 1) / GBM) * ((N + GBN - 1) / GBN);
  int kps = (K + splitk - 1) / splitk;
  kps = (kps + GBK - 1) / GBK * GBK;
  const int S = (K + kps - 1) / kps;
  dim3 grid(tiles, S);
  const bool full = M % GBM == 0 && N % GBN == 0 && K % kps == 0 && kps % GBK == 0;
#define GEMM_LAUNCH(SPL, CHK, RED)                                                            \
  gemm_bf16_kernel<SPL, CHK, RED><<<grid, 256, 0, st>>>((const bf16*)X, (const bf16*)W,         \
                                                        (bf16*)Y, ws, M, N, K, ldx, ldw, ldy,  \
                                                        kps, counters)
  if (S == 1) {
    if (full) GEMM_LAUNCH(false, false, false); else GEMM_LAUNCH(false, true, false);
  } else if (counters != nullptr && N % 4 == 0) {
    // split-K combined inside the launch by each tile's last-arriving slice
    if (full) GEMM_LAUNCH(true, false, true); else GEMM_LAUNCH(true, true, true);
  } else {
    if (full) GEMM_LAUNCH(true, false, false); else GEMM_LAUNCH(true, true, false);
    long blocks = ((long)M * N / 4 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    splitk_reduce_kernel<<<(int)blocks, 256, 0, st>>>(ws, (bf16*)Y, S, M, N, ldy);
  }
#undef GEMM_LAUNCH
}

}  // namespace akap
