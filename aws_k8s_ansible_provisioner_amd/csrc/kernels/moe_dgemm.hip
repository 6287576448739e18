// Grouped expert GEMM for MoE decode on gfx950 (Mixtral 8x7B: every expert's weights are
// streamed every step, ~2.8 GB per layer, so the kernel must run at the HBM rate).
//
//   Y[r] = A[row(r)] . W[e(tile(r))]^T     r over the expert-sorted, block-padded rows
//
// Tile = BM (32 | 64) rows x 128 columns, one expert per tile; the host picks BM from the
// expected rows per expert (T*top_k/E) so one tile usually covers an expert: a second tile
// of the same expert re-streams its weights, a half-empty tile wastes MFMA work only.  The wide N tile keeps the
// re-read activation traffic at 1/4 of the weight bytes (a 64x64 tile reads as many
// activation bytes as weight bytes through each CU's load path).  4 waves, wave w owns
// columns [32w, 32w+32) of the tile (2x2 v_mfma_f32_16x16x32_bf16), BK = 64, full-line
// staging (8 lanes per 128-B row), PF k-tiles of loads in flight in registers (the
// compile-time ring of dgemm.hip), XOR-swizzled LDS double buffer.
//
//   GATHER   row(r) = sorted_ids[r] / top_k (hidden-state rows; padding rows read row 0 and
//            their outputs are never combined), else row(r) = r
//   SILU     W = [gate; up] (N = 2F) read gate/up-interleaved in 16-row groups (dgemm.hip
//            EPI_SILU): Y[r, f] = bf16(bf16(silu(g)) * u), Y is [rows, F] -- the SwiGLU of
//            the expert FFN happens in the w13 GEMM's epilogue.
#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int MBN = 128, MBK = 64;

__device__ __forceinline__ int mswz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }

// BM = rows per tile (32 or 64): 4 waves as WM (= BM/32) x WN (= 4/WM), each owning a
// 32-row x (128/WN)-col sub-tile = 2 x JN 16x16 MFMA tiles.
// SPLIT: K is split over gridDim.z; each slice writes fp32 partials P[z, row, col] (ldy = N)
// that moe_combine_split_kernel sums while combining (no extra launch).
template <int BM, bool GATHER, bool SILU, int PF, bool SPLIT, bool NTW = false>
__global__ __launch_bounds__(256, 2) void moe_dgemm_kernel(const bf16* __restrict__ A,
                                                           const bf16* __restrict__ W,
                                                           bf16* __restrict__ Y,
                                                           float* __restrict__ P,
                                                           const int32_t* __restrict__ sorted_ids,
                                                           const int32_t* __restrict__ tile_expert,
                                                           int n_flat, int topk, int N, int K,
                                                           int lda, int ldy, int rows) {
  constexpr int WM = BM / 32, WN = 4 / WM, WCOLS = MBN / WN, JN = WCOLS / 16;
  constexpr int AR = BM / 32;  // A rows staged per thread
  // one __shared__ object: [buf 2][A BM rows | W 128 rows][8 chunks] bf16x8
  __shared__ bf16x8 lds[2 * (BM + MBN) * 8];
  const int tile = blockIdx.x;
  const int e = tile_expert[tile];
  if (e < 0) return;  // past the padded row count (graph-safe fixed grid); uniform exit
  const int m0 = tile * BM, n0 = blockIdx.y * MBN;
  const int kps = K / gridDim.z, kbeg = blockIdx.z * kps;  // host: kps % (MBK * PF) == 0
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int fr = lane & 15, fg = lane >> 4;
  const int s_ch = tid & 7, s_r = tid >> 3;  // staging chunk / row (0..31)

  const bf16* xa[AR];
#pragma unroll
  for (int c = 0; c < AR; ++c) {
    int arow = m0 + s_r + 32 * c;
    if constexpr (GATHER) {
      const int sid = sorted_ids[arow];
      arow = sid < n_flat ? sid / topk : 0;
    }
    xa[c] = A + (size_t)arow * lda;
  }
  const bf16* wb[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int v = n0 + s_r + 32 * c;  // virtual column
    int wrow = v < N ? v : 0;
    if constexpr (SILU) wrow = v < N ? ((v >> 4) & 1) * (N >> 1) + (v >> 5) * 16 + (v & 15) : 0;
    wb[c] = W + ((size_t)e * N + wrow) * K;
  }

  bf16x8 sa[PF][AR], sb[PF][4];
  auto gload = [&](int q, int k0) {
    const int kk = k0 + s_ch * 8;
#pragma unroll
    for (int c = 0; c < AR; ++c) sa[q][c] = *reinterpret_cast<const bf16x8*>(xa[c] + kk);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bf16x8* src = reinterpret_cast<const bf16x8*>(wb[c] + kk);
      sb[q][c] = NTW ? __builtin_nontemporal_load(src) : *src;
    }
  };
  constexpr int BUF = (BM + MBN) * 8;
  auto sstore = [&](int q, int buf) {
#pragma unroll
    for (int c = 0; c < AR; ++c) lds[buf * BUF + mswz(s_r + 32 * c, s_ch)] = sa[q][c];
#pragma unroll
    for (int c = 0; c < 4; ++c) lds[buf * BUF + BM * 8 + mswz(s_r + 32 * c, s_ch)] = sb[q][c];
  };
  f32x4 acc[2][JN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma = [&](int buf) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[2], bfr[JN];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = lds[buf * BUF + mswz(wm * 32 + i * 16 + fr, ks * 4 + fg)];
#pragma unroll
      for (int j = 0; j < JN; ++j)
        bfr[j] = lds[buf * BUF + BM * 8 + mswz(wn * WCOLS + j * 16 + fr, ks * 4 + fg)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = kps / MBK;
#pragma unroll
  for (int q = 0; q < PF; ++q) gload(q, kbeg + q * MBK);
  int t = 0;
  for (; t + PF < nk; t += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int buf = (t + q) & 1;
      sstore(q, buf);
      __syncthreads();
      gload(q, kbeg + (t + q + PF) * MBK);
      __builtin_amdgcn_sched_barrier(0);  // keep the refill here (see dgemm.hip)
      mfma(buf);
    }
  }
#pragma unroll
  for (int q = 0; q < PF; ++q) {
    const int buf = (t + q) & 1;
    sstore(q, buf);
    __syncthreads();
    mfma(buf);
  }

  // epilogue: lane holds rows wm*32 + i*16 + fg*4 + r, column fr of each 16-col sub-tile j
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm * 32 + i * 16 + fg * 4 + r;
      if constexpr (SILU) {
#pragma unroll
        for (int jj = 0; jj < JN / 2; ++jj) {  // sub-tiles 2jj / 2jj+1 = gate / up
          const int vb = n0 + wn * WCOLS + 32 * jj;
          if (vb + 16 + fr < N) {
            const float g = bf2f(f2bf(acc[i][2 * jj][r]));
            const float u = bf2f(f2bf(acc[i][2 * jj + 1][r]));
            const float sg = bf2f(f2bf(g / (1.f + __expf(-g))));
            Y[(size_t)row * ldy + (vb >> 1) + fr] = f2bf(sg * u);
          }
        }
      } else if constexpr (SPLIT) {
        float* pz = P + ((size_t)blockIdx.z * rows + row) * N;
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int col = n0 + wn * WCOLS + j * 16 + fr;
          if (col < N) pz[col] = acc[i][j][r];
        }
      } else {
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int col = n0 + wn * WCOLS + j * 16 + fr;
          if (col < N) Y[(size_t)row * ldy + col] = f2bf(acc[i][j][r]);
        }
      }
    }
}

bool moe_dgemm_supported(int N, int K, int pf, int silu, int splitk) {
  if (pf != 1 && pf != 2 && pf != 4) return false;
  if (splitk < 1 || K % splitk || (K / splitk) % (MBK * pf)) return false;
  if (silu && splitk > 1) return false;
  return silu ? N % 32 == 0 : N % 8 == 0;
}

// out[t] = sum_k w[t,k] * sum_z P[z, inv[t*K+k]]  (fp32 partial slices of the down GEMM)
__global__ __launch_bounds__(256) void moe_combine_split_kernel(const float* __restrict__ P,
                                                                const float* __restrict__ wts,
                                                                const int32_t* __restrict__ inv,
                                                                bf16* __restrict__ out, int T,
                                                                int topk, int d, int S,
                                                                int rows) {
  const int vpr = d / 8;
  const long total = (long)T * vpr;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    int t, c;  // 32-bit split when it fits (no 64-bit division per element)
    if (total < (1L << 30)) {
      t = (int)i / vpr;
      c = ((int)i - t * vpr) * 8;
    } else {
      t = (int)(i / vpr);
      c = (int)(i % vpr) * 8;
    }
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < topk; ++k) {
      const int pos = inv[(size_t)t * topk + k];
      if (pos < 0) continue;  // skipped (expert-parallel padding) row
      const float wk = wts[(size_t)t * topk + k];
      const size_t r = (size_t)pos;
      for (int z = 0; z < S; ++z) {
        const f32x4* p = reinterpret_cast<const f32x4*>(P + ((size_t)z * rows + r) * d + c);
        const f32x4 a = p[0], b = p[1];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[j] += wk * a[j];
          acc[4 + j] += wk * b[j];
        }
      }
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    *reinterpret_cast<bf16x8*>(out + (size_t)t * d + c) = o;
  }
}

void launch_moe_combine_split(const float* P, const float* wts, const int32_t* inv, void* out,
                              int T, int topk, int d, int S, int rows, hipStream_t s) {
  if (T == 0) return;
  long blocks = ((long)T * (d / 8) + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  moe_combine_split_kernel<<<(int)blocks, 256, 0, s>>>(P, wts, inv, (bf16*)out, T, topk, d, S,
                                                       rows);
}

template <int BM, bool G, bool S, bool SPL>
static void moe_dgemm_pf(dim3 grid, int pf, bool ntw, hipStream_t s, const bf16* A, const bf16* W, bf16* Y,
                         float* P, const int32_t* sid, const int32_t* te, int n_flat, int topk,
                         int N, int K, int lda, int ldy, int rows) {
#define MOE_L(PFV, NT) moe_dgemm_kernel<BM, G, S, PFV, SPL, NT><<<grid, 256, 0, s>>>( \
      A, W, Y, P, sid, te, n_flat, topk, N, K, lda, ldy, rows)
  switch (pf) {
    case 4: if (ntw) MOE_L(4, true); else MOE_L(4, false); break;
    case 2: if (ntw) MOE_L(2, true); else MOE_L(2, false); break;
    default: MOE_L(1, false);
  }
#undef MOE_L
}

template <int BM>
static void moe_dgemm_bm(dim3 grid, int gather, int silu, int pf, bool ntw, hipStream_t s, const bf16* a,
                         const bf16* w, bf16* y, float* P, const int32_t* sid, const int32_t* te,
                         int n_flat, int topk, int N, int K, int lda, int ldy, int rows) {
  const bool spl = grid.z > 1;
  if (gather && silu)
    moe_dgemm_pf<BM, true, true, false>(grid, pf, ntw, s, a, w, y, P, sid, te, n_flat, topk, N, K, lda, ldy, rows);
  else if (silu)
    moe_dgemm_pf<BM, false, true, false>(grid, pf, ntw, s, a, w, y, P, sid, te, n_flat, topk, N, K, lda, ldy, rows);
  else if (gather && spl)
    moe_dgemm_pf<BM, true, false, true>(grid, pf, ntw, s, a, w, y, P, sid, te, n_flat, topk, N, K, lda, ldy, rows);
  else if (gather)
    moe_dgemm_pf<BM, true, false, false>(grid, pf, ntw, s, a, w, y, P, sid, te, n_flat, topk, N, K, lda, ldy, rows);
  else if (spl)
    moe_dgemm_pf<BM, false, false, true>(grid, pf, ntw, s, a, w, y, P, sid, te, n_flat, topk, N, K, lda, ldy, rows);
  else
    moe_dgemm_pf<BM, false, false, false>(grid, pf, ntw, s, a, w, y, P, sid, te, n_flat, topk, N, K, lda, ldy, rows);
}

void launch_moe_dgemm(const void* A, const void* W, void* Y, const int32_t* sorted_ids,
                      const int32_t* tile_expert, int max_tiles, int n_flat, int topk, int N,
                      int K, int lda, int ldy, int gather, int silu, int pf, int bm, int splitk,
                      float* partials, bool ntw, hipStream_t s) {
  if (max_tiles == 0) return;
  dim3 grid(max_tiles, (N + MBN - 1) / MBN, splitk);
  const bf16* a = (const bf16*)A;
  const bf16* w = (const bf16*)W;
  bf16* y = (bf16*)Y;
  const int rows = max_tiles * bm;
  if (bm == 64)
    moe_dgemm_bm<64>(grid, gather, silu, pf, ntw, s, a, w, y, partials, sorted_ids, tile_expert, n_flat, topk, N, K, lda, ldy, rows);
  else
    moe_dgemm_bm<32>(grid, gather, silu, pf, ntw, s, a, w, y, partials, sorted_ids, tile_expert, n_flat, topk, N, K, lda, ldy, rows);
}

}  // namespace akap
