// Prefill / large-M GEMM for gfx950:  Y[M,N] = X[M,K] . W[N,K]^T  (bf16 in, fp32 accumulate),
// dense or expert-grouped, optional SwiGLU epilogue.  The chunked-prefill projections
// (M = thousands of tokens) and the MoE expert GEMMs of a prefill chunk run here.
//
// Tile: 256 x 256 outputs per 512-thread workgroup (8 waves as 2 (M) x 4 (N), 128 x 64 per
// wave = 8 x 4 MFMA 16x16x32 fragments, 128 accumulator VGPRs), K in 64-deep tiles through two
// 64 KB LDS buffers filled by buffer_load_dwordx4 ... lds (LDS-DMA through SGPR buffer
// descriptors: 32-bit per-lane offsets, X rows past M read as 0).  The K loop is cut into four
// PHASES per K tile; each computes one 64 x 32 quadrant of the wave's outputs (16 MFMAs).  A
// "half-tile" is 128 rows x 64 k (16 KB: two 1-KiB DMA instructions per wave), issued in the
// order the phases consume them, so every wait is a counted `s_waitcnt vmcnt` (never 0 in
// steady state: cdna_hip_programming.md "Pipelining across barriers", T3+T4).
// NB = 2 (plain store; two raw s_barriers per K tile):
//   phase | counted wait + barrier           | ds_reads issued            | DMA issued
//   1     | W right + A bottom of tile t     | B right + A bottom (t)     | W right, A bottom (t+1)
//   2     | --                               | --                         | --
//   3     | --                               | --                         | A top (t+2)
//   4     | A top + W left of t+1            | A top + B left (t+1)       | W left (t+2)
// NB = 4 (SwiGLU epilogue: reading both fragment sets in phase 1 would spill there) adds a
// barrier to phases 2 and 3 and reads A bottom in phase 2.  WAR safety: a half-tile region is
// re-filled only after the barrier that follows its last reads (A top / W left of tile t+2 go
// into buffer t&1 after phase 1 of t, whose barrier retired their phase-4-of-(t-1) reads).
// Fragment reads for the next phases are issued before the current MFMAs, so LDS latency hides
// under them.  One __shared__ array (no second LDS object: the compiler would drain vmcnt in the
// loop, ibid. item 4a), raw s_barrier (never __syncthreads, whose fence drains the DMAs).
// Measured: 0.81-0.86x of hipBLASLt on dense 8B-class shapes, 1.1-3.2x torch._grouped_mm on
// expert-grouped ones (profiles/r4_pgemm_nb_ab.log); deeper rings, one barrier per 32-deep step
// and 4-wave 128 x 128 sub-tiles were slower (r4_pgemm_v2_ring_rejected.log,
// r4_pgemm_variants_pmc.log).
//
// LDS image: 128-B rows (64 bf16 of K), 16-B chunk c of row r stored at chunk c ^ ((r >> 1) & 7):
// for each ds_read_b128 lane group (rows {0-3, 12-15} at chunk c and rows {4-11} at chunk c+1,
// c even) the 16 addresses fall on 16 distinct 16-B bank slots -- conflict-free.  The DMA
// destination is lane-linear, so the XOR goes on the per-lane SOURCE address and on the reads
// (the same involution, cdna_hip_programming.md rule 21).
//
// Operands are swapped in the MFMA (W fragment as A, X fragment as B): the accumulator then
// holds 4 CONSECUTIVE output columns of one row per lane, stored as one 8-byte write.
//
// Grid: XCD-aware (common.h xcd_remap: 32 consecutive logical tiles share an XCD and its L2)
// and grouped rasterisation (8 M-tiles x N-tiles per block, M fastest), so the WGs of one XCD
// stream the same K slices of 8 X panels and 4 W panels together (pg_tile).
// Grouped (MoE): group g owns rows [offs[g-1], offs[g]) of X and weight W + g*N*K; the same
// raster runs over the concatenated list of every group's M tiles; the grid is an upper bound
// (sum of ceil(rows_g / 256) <= ceil(M / 256) + G) and surplus WGs exit.
// SwiGLU epilogue (EPI_SILU): W rows are the [gate; up] halves of a [2F, K] weight; tile column
// v reads weight row ((v >> 4) & 1) * F + (v >> 5) * 16 + (v & 15) (the gdgemm.hip mapping), so
// gate and up of one output column land in the same lane of adjacent fragments and the kernel
// writes act[M, F] = silu(gate) * up directly.
#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int PG_T = 256;        // tile rows / cols
constexpr int PG_BK = 64;        // K tile
constexpr int PG_THREADS = 512;  // 8 waves
constexpr int PG_BUF = 2 * PG_T * 8;  // 16-B units per LDS buffer (A 256 rows + W 256 rows)

__device__ __forceinline__ int pg_unit(int row, int chunk) {
  return row * 8 + (chunk ^ ((row >> 1) & 7));
}

__device__ __forceinline__ void pg_glds(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0,
                                   0);
}

// LDS hand-off point: every wave's ds_reads of the previous phase retired, then the barrier;
// the empty asm keeps the compiler from hoisting any LDS read above it
__device__ __forceinline__ void pg_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// wait until at most 2 * `later` of this wave's DMA instructions are outstanding
__device__ __forceinline__ void pg_wait(int later) {
  if (later >= 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (later == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (later == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int V>
struct HalfTile {
  static constexpr int value = V;
};
using H0 = HalfTile<0>;  // A rows of the waves' top quadrants
using H1 = HalfTile<1>;  // W rows of the left quadrants
using H2 = HalfTile<2>;  // W rows of the right quadrants
using H3 = HalfTile<3>;  // A rows of the bottom quadrants

// Workgroup -> output tile.  Dense: XCD-aware ids (common.h xcd_remap: 32 consecutive ids per
// XCD) rasterised in blocks of GM M-tiles x all N-tiles, M fastest, so the WGs of one XCD share
// a few X and W panels in its L2.  Grouped (MoE): the same raster over the concatenated list of
// every group's M tiles (group g owns rows [offs[g-1], offs[g]), ceil(rows_g / 256) tiles); the
// grid is the upper bound ceil(M / 256) + G tiles and surplus ids return false (uniform).
template <bool GROUPED>
__device__ __forceinline__ bool pg_tile(const PGemmArgs& p, int& tm, int& tn, int& group,
                                        int& row_lo, int& row_hi) {
  constexpr int GM = 8;
  const int tiles_n = p.N / PG_T;
  const int nwg = gridDim.x;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int tiles_m = nwg / tiles_n;  // dense: exact; grouped: the upper bound
  const int per_block = GM * tiles_n;
  const int first_m = (id / per_block) * GM;
  const int gm = min(tiles_m - first_m, GM);
  const int in = id % per_block;
  int mt = first_m + in % gm;
  tn = in / gm;
  group = 0;
  row_lo = 0;
  row_hi = p.M;
  if constexpr (!GROUPED) {
    tm = mt;
    return true;
  } else {
    int lo = 0;
    for (int g = 0; g < p.groups; ++g) {
      const int hi = min(p.offs[g], p.M);  // offsets past M never store out of bounds
      const int nt = (hi - lo + PG_T - 1) / PG_T;
      if (mt < nt) {
        tm = mt;
        group = g;
        row_lo = lo;
        row_hi = hi;
        return true;
      }
      mt -= nt;
      lo = hi;
    }
    return false;
  }
}

template <int EPI, bool GROUPED, int NB>
__global__ __launch_bounds__(PG_THREADS, 1) void pgemm_kernel(PGemmArgs p) {
  __shared__ bf16x8 lds[2 * PG_BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int fr = lane & 15, fg = lane >> 4;

  // ---- tile of this workgroup --------------------------------------------------------------
  int tm, tn, group, row_lo, row_hi;
  if (!pg_tile<GROUPED>(p, tm, tn, group, row_lo, row_hi)) return;  // surplus WG (uniform)
  const int m0 = row_lo + tm * PG_T, n0 = tn * PG_T;
  const int nk = p.K / PG_BK;
  const bf16* X = static_cast<const bf16*>(p.X);
  const bf16* W = static_cast<const bf16*>(p.W) + (GROUPED ? (size_t)group * p.N * p.K : 0);

  // ---- per-lane DMA sources: half-tile h (0 A top, 1 W left, 2 W right, 3 A bottom), the
  // wave's two 8-row pieces q = 2w, 2w+1 of it.  Rows past the tile's valid range re-read a
  // valid row (results never stored).
  // DMA through buffer resources (buffer_load_dwordx4 ... lds): SGPR descriptors for X and W,
  // 32-bit per-lane byte offsets (8 VGPRs for the 8 sources), the K position in the scalar
  // offset.  X rows past M fall outside the descriptor's range and read as 0 (rows of a
  // neighbouring group inside it are harmless: those accumulator rows are never stored).
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)X, (short)0, (int)((size_t)p.M * p.ldx * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)W, (short)0, (int)((size_t)p.N * p.K * 2), 0x00020000);
  uint32_t voff[4][2];
  int dst[4][2];  // 16-B unit offset inside a buffer
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int q = 2 * w + e;
      int r0;
      if (h == 0) r0 = (q >> 3) * 128 + (q & 7) * 8;
      else if (h == 3) r0 = (q >> 3) * 128 + 64 + (q & 7) * 8;
      else if (h == 1) r0 = (q >> 2) * 64 + (q & 3) * 8;
      else r0 = (q >> 2) * 64 + 32 + (q & 3) * 8;
      const int row = r0 + (lane >> 3);
      const int chunk = (lane & 7) ^ ((row >> 1) & 7);
      if (h == 0 || h == 3) {
        voff[h][e] = (uint32_t)(((m0 + row) * p.ldx + chunk * 8) * 2);
        dst[h][e] = r0 * 8;
      } else {
        const int v = n0 + row;
        int wr = v;
        if constexpr (EPI == EPI_SILU) wr = ((v >> 4) & 1) * (p.N >> 1) + (v >> 5) * 16 + (v & 15);
        voff[h][e] = (uint32_t)((wr * p.K + chunk * 8) * 2);
        dst[h][e] = PG_T * 8 + r0 * 8;
      }
    }
  // half-tile seq s = 4 j + h (tile j, h in consumption order A top, W left, W right, A bottom);
  // every call site names h at compile time (no dynamic register indexing)
  auto issue = [&](auto hc, int j) {
    constexpr int h = decltype(hc)::value;
    if (j >= nk) return;
    bf16x8* buf = lds + (j & 1) * PG_BUF;
    const uint32_t kb = (uint32_t)(j * PG_BK * 2);
#pragma unroll
    for (int e = 0; e < 2; ++e)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          h == 0 || h == 3 ? rx : rw, (__attribute__((address_space(3))) void*)(buf + dst[h][e]),
          16, voff[h][e], kb, 0, 0);
  };
  auto later = [&](int s) { return min(3, 4 * nk - 1 - s); };

  // ---- fragments -----------------------------------------------------------------------------
  bf16x8 at[4][2], ab[4][2], bl[2][2], br[2][2];
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto rd_a = [&](bf16x8 (&a)[4][2], const bf16x8* buf, int half) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        a[i][s] = buf[pg_unit(wm * 128 + half * 64 + i * 16 + fr, fg + 4 * s)];
  };
  auto rd_b = [&](bf16x8 (&b)[2][2], const bf16x8* buf, int half) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        b[j][s] = buf[PG_T * 8 + pg_unit(wn * 64 + half * 32 + j * 16 + fr, fg + 4 * s)];
  };
  auto mma = [&](const bf16x8 (&a)[4][2], const bf16x8 (&b)[2][2], int i0, int j0) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i0 + i][j0 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][s], a[i][s], acc[i0 + i][j0 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- prologue: half-tiles 0..5 in flight, tile 0's A top + W left in registers -------------
  issue(H0{}, 0);
  issue(H1{}, 0);
  issue(H2{}, 0);
  issue(H3{}, 0);
  issue(H0{}, 1);
  issue(H1{}, 1);
  {
    const int outstanding = min(6, 4 * nk) - 2;  // half-tiles after seq 1 already issued
    if (outstanding >= 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // nk == 1: seqs 2, 3 after it
  }
  pg_sync();
  rd_a(at, lds, 0);
  rd_b(bl, lds, 0);

  // outstanding half-tiles allowed while waiting for seq s when seqs <= last were issued
  auto allow = [&](int s, int last) { return max(0, min(last, 4 * nk - 1) - s); };
  for (int t = 0; t < nk; ++t) {
    const bf16x8* cur = lds + (t & 1) * PG_BUF;
    const bf16x8* nxt = lds + ((t + 1) & 1) * PG_BUF;
    if constexpr (NB == 4) {
      // phase 1: W right of t landed -> its fragments; DMA W right (t+1); quadrant top x left
      pg_wait(later(4 * t + 2));
      pg_sync();
      rd_b(br, cur, 1);
      issue(H2{}, t + 1);
      mma(at, bl, 0, 0);
      // phase 2: A bottom of t -> fragments; DMA A bottom (t+1); quadrant top x right
      pg_wait(later(4 * t + 3));
      pg_sync();
      rd_a(ab, cur, 1);
      issue(H3{}, t + 1);
      mma(at, br, 0, 2);
      // phase 3: buffer t&1 fully read -> DMA A top (t+2) into it; quadrant bottom x left
      pg_sync();
      issue(H0{}, t + 2);
      mma(ab, bl, 4, 0);
    } else {
      // phase 1: W right + A bottom of t landed -> both fragment sets; DMA both for t+1
      pg_wait(allow(4 * t + 3, 4 * t + 5));
      pg_sync();
      rd_b(br, cur, 1);
      rd_a(ab, cur, 1);
      issue(H2{}, t + 1);
      issue(H3{}, t + 1);
      mma(at, bl, 0, 0);
      // phase 2 (no barrier): quadrant top x right
      mma(at, br, 0, 2);
      // phase 3 (no barrier): A top of t+2 into buffer t&1 -- its last reads (phase 4 of t-1)
      // retired before phase 1's barrier; quadrant bottom x left
      issue(H0{}, t + 2);
      mma(ab, bl, 4, 0);
    }
    // phase 4: A top + W left of t+1 -> fragments; DMA W left (t+2); quadrant bottom x right
    if (t + 1 < nk) {
      if constexpr (NB == 4) pg_wait(later(4 * (t + 1) + 1));
      else pg_wait(allow(4 * t + 5, 4 * t + 8));
      pg_sync();
      rd_a(at, nxt, 0);
      rd_b(bl, nxt, 0);
    }
    issue(H1{}, t + 2);
    mma(ab, br, 4, 2);
  }

  // ---- epilogue: lane holds rows wm*128 + i*16 + fr, 4 consecutive cols per fragment ---------
  bf16* Y = static_cast<bf16*>(p.Y);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wm * 128 + i * 16 + fr;
    if (row >= row_hi) continue;
    if constexpr (EPI == EPI_SILU) {
      // fragments j (gate) and j+1 (up) of one 32-column group -> 16 output columns
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int col = (n0 >> 1) + wn * 32 + jj * 16 + fg * 4;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float g = bf2f(f2bf(acc[i][2 * jj][r]));
          const float u = bf2f(f2bf(acc[i][2 * jj + 1][r]));
          o[r] = f2bf(bf2f(f2bf(g / (1.f + __expf(-g)))) * u);
        }
        *reinterpret_cast<bf16x4*>(Y + (size_t)row * p.ldy + col) = o;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn * 64 + j * 16 + fg * 4;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r]);
        *reinterpret_cast<bf16x4*>(Y + (size_t)row * p.ldy + col) = o;
      }
    }
  }
}

bool pgemm_supported(int M, int N, int K) {
  return M > 0 && N > 0 && N % PG_T == 0 && K >= PG_BK && K % PG_BK == 0;
}

void launch_pgemm(const PGemmArgs& p, int epi, hipStream_t st) {
  if (p.M == 0) return;
  const int tiles_n = p.N / PG_T;
  const int grid = p.groups > 0 ? ((p.M + PG_T - 1) / PG_T + p.groups) * tiles_n
                                 : ((p.M + PG_T - 1) / PG_T) * tiles_n;
  // two barriers per K tile (measured 1-4 % faster than four, profiles/r4_pgemm_nb_ab.log); the
  // SwiGLU form keeps four: with both fragment sets read in phase 1 it would spill
  if (p.groups > 0) {
    if (epi == EPI_SILU) pgemm_kernel<EPI_SILU, true, 4><<<grid, PG_THREADS, 0, st>>>(p);
    else pgemm_kernel<EPI_STORE, true, 2><<<grid, PG_THREADS, 0, st>>>(p);
  } else {
    if (epi == EPI_SILU) pgemm_kernel<EPI_SILU, false, 4><<<grid, PG_THREADS, 0, st>>>(p);
    else pgemm_kernel<EPI_STORE, false, 2><<<grid, PG_THREADS, 0, st>>>(p);
  }
}

}  // namespace akap
