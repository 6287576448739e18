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
// DEFAULT K loop (SCHED 4, "stream-first", round 6): one counted wait + one barrier per K tile,
// then the whole next K tile (four half-tiles, 64 KiB) is requested at once and streams into the
// other buffer under this tile's 64 MFMAs per wave.  A no-math probe of exactly this operand
// stream runs as fast as hipBLASLt's whole GEMM, and the phase pipeline below measured ~stream +
// math; the stream-first loop is 5-14 % faster than it (0.70-0.88x hipBLASLt dense, 0.97-1.11x
// with the SwiGLU epilogue, profiles/r6_pgemm_isa_diff.md).  The phase pipeline (SCHED 1):
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
#include <cstdlib>

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

// wait until at most P * `later` of this wave's DMA instructions are outstanding (P = DMA
// pieces per half-tile per wave: 2 with 8 waves, 4 with 4 waves)
template <int P>
__device__ __forceinline__ void pg_wait(int later) {
  if (later >= 6) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * P) : "memory");
  else if (later == 5) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * P) : "memory");
  else if (later == 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * P) : "memory");
  else if (later == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * P) : "memory");
  else if (later == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * P) : "memory");
  else if (later == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Wave geometry of the 256 x 256 tile: WAVES = 8 -> 2 (M) x 4 (N) waves of 128 x 64 outputs;
// WAVES = 4 -> 2 x 2 waves of 128 x 128 (one wave per SIMD: 64 accumulator fragments = 256
// accumulator registers, a third fewer LDS fragment reads per MFMA).  Each wave's rows split
// into a top and a bottom 64-row half, its columns into a left and a right half, so both forms
// run the same four-quadrant phase pipeline over the same four half-tiles.
template <int WAVES>
struct PgGeo {
  static constexpr int THREADS = WAVES * 64;
  static constexpr int P = 16 / WAVES;        // DMA pieces (1 KiB) per half-tile per wave
  static constexpr int WN = WAVES / 2;        // waves along N
  static constexpr int WCOLS = PG_T / WN;     // output columns per wave
  static constexpr int NJ = WCOLS / 32;       // 16-column fragments per column half
};

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
  const int GM = p.gm > 0 ? p.gm : 8;
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

// The 256 x 256 main loop over K tiles [kt0, kt0 + nk): X rows from m0 (rows past the X
// descriptor's range read as 0), W rows of tile columns n0.. (SILU_ROWS: the [gate; up] row
// interleave of the SwiGLU epilogue, `nhalf` = F).  Leaves the tile in acc (lane: rows
// wm*128 + i*16 + fr, 4 consecutive columns wn*64 + j*16 + fg*4 per fragment).
// a wave's accumulator fragments: rows i (8 x 16), columns j (2 NJ x 16)
template <int NJ2>
struct PgAcc {
  f32x4 v[8][NJ2];
};

template <int NB, bool SILU_ROWS, int WAVES, typename ACC, int SCHED = 1>
__device__ __forceinline__ void pg_mainloop(bf16x8* lds, const __amdgpu_buffer_rsrc_t rx,
                                            const __amdgpu_buffer_rsrc_t rw, int ldx, int K,
                                            int nhalf, int m0, int n0, int kt0, int nk,
                                            ACC& accs) {
  using G = PgGeo<WAVES>;
  constexpr int P = G::P, NJ = G::NJ;
  auto& acc = accs.v;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / G::WN, wn = w % G::WN;
  const int fr = lane & 15, fg = lane >> 4;
  // ---- per-lane DMA sources: half-tile h (0 A top, 1 W left, 2 W right, 3 A bottom), the
  // wave's two 8-row pieces q = 2w, 2w+1 of it.  Rows past the tile's valid range re-read a
  // valid row (results never stored).
  // DMA through buffer resources (buffer_load_dwordx4 ... lds): SGPR descriptors for X and W,
  // 32-bit per-lane byte offsets (8 VGPRs for the 8 sources), the K position in the scalar
  // offset.  X rows past M fall outside the descriptor's range and read as 0 (rows of a
  // neighbouring group inside it are harmless: those accumulator rows are never stored).
  uint32_t voff[4][PgGeo<WAVES>::P];
  int dst[4][PgGeo<WAVES>::P];  // 16-B unit offset inside a buffer
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int e = 0; e < P; ++e) {
      const int q = P * w + e;  // the half-tile's 16 pieces of 8 rows
      int r0;
      if (h == 0) r0 = (q >> 3) * 128 + (q & 7) * 8;
      else if (h == 3) r0 = (q >> 3) * 128 + 64 + (q & 7) * 8;
      else if constexpr (WAVES == 8) r0 = (q >> 2) * 64 + (h == 2 ? 32 : 0) + (q & 3) * 8;
      else r0 = (q >> 3) * 128 + (h == 2 ? 64 : 0) + (q & 7) * 8;
      const int row = r0 + (lane >> 3);
      const int chunk = (lane & 7) ^ ((row >> 1) & 7);
      if (h == 0 || h == 3) {
        voff[h][e] = (uint32_t)(((m0 + row) * ldx + chunk * 8) * 2);
        dst[h][e] = r0 * 8;
      } else {
        const int v = n0 + row;
        int wr = v;
        if constexpr (SILU_ROWS) wr = ((v >> 4) & 1) * nhalf + (v >> 5) * 16 + (v & 15);
        voff[h][e] = (uint32_t)((wr * K + chunk * 8) * 2);
        dst[h][e] = PG_T * 8 + r0 * 8;
      }
    }
  // half-tile seq s = 4 j + h (tile j, h in consumption order A top, W left, W right, A bottom);
  // every call site names h at compile time (no dynamic register indexing)
  auto issue = [&](auto hc, int j) {
    constexpr int h = decltype(hc)::value;
    if (j >= nk) return;
    bf16x8* buf = lds + (j & 1) * PG_BUF;
    const uint32_t kb = (uint32_t)((kt0 + j) * PG_BK * 2);
    // (the host pass of hipcc rejects this builtin inside the wave-count template's generic
    // lambda during overload resolution; the device pass compiles it)
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int e = 0; e < PgGeo<WAVES>::P; ++e)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          h == 0 || h == 3 ? rx : rw, (__attribute__((address_space(3))) void*)(buf + dst[h][e]),
          16, voff[h][e], kb, 0, 0);
#endif
  };
  auto later = [&](int s) { return min(3, 4 * nk - 1 - s); };

  // ---- fragments -----------------------------------------------------------------------------
  bf16x8 at[4][2], ab[4][2], bl[PgGeo<WAVES>::NJ][2], br[PgGeo<WAVES>::NJ][2];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2 * NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto rd_a = [&](bf16x8 (&a)[4][2], const bf16x8* buf, int half) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        a[i][s] = buf[pg_unit(wm * 128 + half * 64 + i * 16 + fr, fg + 4 * s)];
  };
  auto rd_b = [&](bf16x8 (&b)[PgGeo<WAVES>::NJ][2], const bf16x8* buf, int half) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        b[j][s] = buf[PG_T * 8 + pg_unit(wn * G::WCOLS + half * (G::WCOLS / 2) + j * 16 + fr,
                                         fg + 4 * s)];
  };
  auto mma = [&](const bf16x8 (&a)[4][2], const bf16x8 (&b)[PgGeo<WAVES>::NJ][2], int i0,
                 int j0) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i0 + i][j0 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][s], a[i][s], acc[i0 + i][j0 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (SCHED == 4) {
    // ---- stream-first schedule: the whole next K tile (all four half-tiles, 64 KiB) is
    // requested right after this tile's barrier and streams under this tile's MFMAs.  The
    // no-math stream of these tiles (one tile in flight, the same pattern) runs as fast as
    // hipBLASLt's whole GEMM, while the phase pipeline above measured stream + math
    // (profiles/r6_pgemm_isa_diff.md, "no-math stream").  One wait, one barrier per K tile.
    issue(H0{}, 0);
    issue(H1{}, 0);
    issue(H2{}, 0);
    issue(H3{}, 0);
    for (int t = 0; t < nk; ++t) {
      const bf16x8* cur = lds + (t & 1) * PG_BUF;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t landed (the only one in flight)
      pg_sync();  // every wave's pieces of t landed; every read of tile t-1 (slot of t+1) retired
      issue(H0{}, t + 1);
      issue(H1{}, t + 1);
      issue(H2{}, t + 1);
      issue(H3{}, t + 1);
      rd_a(at, cur, 0);
      rd_b(bl, cur, 0);
      rd_b(br, cur, 1);
      rd_a(ab, cur, 1);
      mma(at, bl, 0, 0);
      mma(at, br, 0, NJ);
      mma(ab, bl, 4, 0);
      mma(ab, br, 4, NJ);
    }
    return;
  }
  if constexpr (SCHED == 2) {
    // ---- early-issue schedule: every half-tile goes out as soon as its slot's previous
    // reads retired -- A top / W left of tile t+2 right after phase 1's barrier of tile t
    // (their slot's last reads were phase 4 of t-1), W right / A bottom of t+2 right after
    // phase 4's barrier of t (last reads: phase 1 of t).  Issue order stays the consumption
    // order (seq 4 j + h), so every wait is still a counted in-order vmcnt, and each
    // half-tile is requested 1.25-1.75 tiles ahead (1.0-1.25 in the schedule below).
    issue(H0{}, 0);
    issue(H1{}, 0);
    issue(H2{}, 0);
    issue(H3{}, 0);
    issue(H0{}, 1);
    issue(H1{}, 1);
    issue(H2{}, 1);
    issue(H3{}, 1);
    auto out = [&](int need, int last) { return max(0, min(last, 4 * nk - 1) - need); };
    pg_wait<P>(out(1, 7));
    pg_sync();
    rd_a(at, lds, 0);
    rd_b(bl, lds, 0);
    for (int t = 0; t < nk; ++t) {
      const bf16x8* cur = lds + (t & 1) * PG_BUF;
      const bf16x8* nxt = lds + ((t + 1) & 1) * PG_BUF;
      // phase 1: W right + A bottom of t landed (seq 4t+3; issued through 4t+7)
      pg_wait<P>(out(4 * t + 3, 4 * t + 7));
      pg_sync();
      rd_b(br, cur, 1);
      if constexpr (NB == 4) {
        issue(H0{}, t + 2);
        issue(H1{}, t + 2);
        mma(at, bl, 0, 0);
        pg_sync();  // (SwiGLU form: A bottom read after a barrier, as below)
        rd_a(ab, cur, 1);
        mma(at, br, 0, NJ);
        pg_sync();
        mma(ab, bl, 4, 0);
      } else {
        rd_a(ab, cur, 1);
        issue(H0{}, t + 2);
        issue(H1{}, t + 2);
        mma(at, bl, 0, 0);
        mma(at, br, 0, NJ);
        mma(ab, bl, 4, 0);
      }
      // phase 4: A top + W left of t+1 (seq 4t+5; issued through 4t+9)
      if (t + 1 < nk) {
        pg_wait<P>(out(4 * t + 5, 4 * t + 9));
        pg_sync();
        rd_a(at, nxt, 0);
        rd_b(bl, nxt, 0);
      } else {
        pg_sync();
      }
      issue(H2{}, t + 2);
      issue(H3{}, t + 2);
      mma(ab, br, 4, NJ);
    }
    return;
  }

  // ---- prologue: half-tiles 0..5 in flight, tile 0's A top + W left in registers -------------
  issue(H0{}, 0);
  issue(H1{}, 0);
  issue(H2{}, 0);
  issue(H3{}, 0);
  issue(H0{}, 1);
  issue(H1{}, 1);
  {
    const int outstanding = min(6, 4 * nk) - 2;  // half-tiles after seq 1 already issued
    if (outstanding >= 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * P) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * P) : "memory");  // nk == 1: seqs 2, 3
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
      pg_wait<P>(later(4 * t + 2));
      pg_sync();
      rd_b(br, cur, 1);
      issue(H2{}, t + 1);
      mma(at, bl, 0, 0);
      // phase 2: A bottom of t -> fragments; DMA A bottom (t+1); quadrant top x right
      pg_wait<P>(later(4 * t + 3));
      pg_sync();
      rd_a(ab, cur, 1);
      issue(H3{}, t + 1);
      mma(at, br, 0, NJ);
      // phase 3: buffer t&1 fully read -> DMA A top (t+2) into it; quadrant bottom x left
      pg_sync();
      issue(H0{}, t + 2);
      mma(ab, bl, 4, 0);
    } else {
      // phase 1: W right + A bottom of t landed -> both fragment sets; DMA both for t+1
      pg_wait<P>(allow(4 * t + 3, 4 * t + 5));
      pg_sync();
      rd_b(br, cur, 1);
      rd_a(ab, cur, 1);
      issue(H2{}, t + 1);
      issue(H3{}, t + 1);
      mma(at, bl, 0, 0);
      // phase 2 (no barrier): quadrant top x right
      mma(at, br, 0, NJ);
      // phase 3 (no barrier): A top of t+2 into buffer t&1 -- its last reads (phase 4 of t-1)
      // retired before phase 1's barrier; quadrant bottom x left
      issue(H0{}, t + 2);
      mma(ab, bl, 4, 0);
    }
    // phase 4: A top + W left of t+1 -> fragments; DMA W left (t+2); quadrant bottom x right
    if (t + 1 < nk) {
      if constexpr (NB == 4) pg_wait<P>(later(4 * (t + 1) + 1));
      else pg_wait<P>(allow(4 * t + 5, 4 * t + 8));
      pg_sync();
      rd_a(at, nxt, 0);
      rd_b(bl, nxt, 0);
    }
    issue(H1{}, t + 2);
    mma(ab, br, 4, NJ);
  }
}

// ------------------------------------------------------------------------------------------
// SCHED 3: the unit-pipelined 4-wave body (built from the ISA of the library kernel that wins
// the prefill shapes, hipBLASLt's MT256x256x64_MI16x16x1 "SK3" kernel: 4 waves of 128 x 128,
// one wave per SIMD, 256 accumulators, every LDS fragment read and every LDS-DMA piece issued
// BETWEEN MFMAs, 3 vmcnt waits and ~2 barriers per 64-deep K tile; profiles/
// r6_pgemm_isa_diff.md).  Against the phase pipeline above (same tile, same waves) it drops:
//   * runtime-selected waits (pg_wait's if-chain: s_cbranch + SALU per wait),
//   * bursts of 16-24 fragment reads before the MFMAs that consume them one by one,
//   * the four-quadrant split of the accumulators (a quadrant's 16 MFMAs per phase).
// Unit u = 32 K columns of the 256 x 256 tile (A 256 rows x 64 B + W 256 rows x 64 B = 32 KiB,
// 8 1-KiB LDS-DMA pieces per wave) in LDS slot u % 4 (128 KiB).  Iteration u:
//   wait unit u+1 landed (vmcnt(16): units u+2, u+3 stay in flight) + lgkmcnt(0) (this wave's
//   fragments of u are in registers), barrier (every wave's are -> slot u % 4 is free);
//   64 MFMAs of unit u on register set u & 1, with the 8 DMA pieces of unit u + 4 (into slot
//   u % 4) and the 16 fragment reads of unit u + 1 (set (u + 1) & 1) interleaved between them
//   (sched_group_barrier: per 8 MFMAs 2 reads and 1 DMA piece).
// One barrier per 32-deep unit; every unit is requested 3 units (1.5 K tiles) ahead.
// LDS rows are 64 B (4 chunks); chunk c of row r is stored at c ^ g((r >> 2) & 3), g = {0, 2,
// 3, 1}: for every ds_read_b128 lane group the 16 (row, chunk) pairs of a 16 x 32 fragment
// read land on 16 distinct 16-B bank slots (conflict-free; derivation in the r6 profile).
constexpr int PU_SLOT = 2 * PG_T * 4;  // 16-B units per slot: A 256 rows + W 256 rows x 4

__device__ __forceinline__ int pu_swz(int row, int c) {
  return c ^ ((0x1320 >> (4 * ((row >> 2) & 3))) & 3);
}

template <bool SILU_ROWS, typename ACC>
__device__ __forceinline__ void pg_mainloop_u(bf16x8* lds, const __amdgpu_buffer_rsrc_t rx,
                                              const __amdgpu_buffer_rsrc_t rw, int ldx, int K,
                                              int nhalf, int m0, int n0, int ku0, int nu,
                                              int st0, ACC& accs) {
  auto& acc = accs.v;  // [8][8]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int fr = lane & 15, fg = lane >> 4;
  // ---- DMA sources: piece e (0..7) of this wave: e < 4 -> A rows (4w+e)*16.., else W rows
  uint32_t voff[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int r16 = (e & 3) + 4 * w;  // which 16-row block of A (e < 4) or W (e >= 4)
    const int row = r16 * 16 + (lane >> 2);
    const int c = pu_swz(row, lane & 3);  // logical chunk held by this lane's LDS slot
    if (e < 4) {
      voff[e] = (uint32_t)(((m0 + row) * ldx + c * 8) * 2);
    } else {
      const int v = n0 + row;
      int wr = v;
      if constexpr (SILU_ROWS) wr = ((v >> 4) & 1) * nhalf + (v >> 5) * 16 + (v & 15);
      voff[e] = (uint32_t)((wr * K + c * 8) * 2);
    }
  }
  auto dma = [&](int u, int e) {  // piece e of unit u into slot u % 4
    bf16x8* slot = lds + (u & 3) * PU_SLOT;
    const int r16 = (e & 3) + 4 * w;
    bf16x8* dst = slot + (e < 4 ? 0 : PG_T * 4) + r16 * 64;
    // units past the end are issued too (no branch in the pipelined body) with a scalar
    // offset past every descriptor's range: the buffer unit drops them without a memory
    // access (the slot they land in is never read again)
    // st0: this workgroup's K start ("StaggerU"): units are visited from st0, wrapping, so
    // workgroups sharing an operand panel do not request the same lines at the same time
    int ku = u + st0;
    if (ku >= nu) ku -= nu;
    const uint32_t kb = u < nu ? (uint32_t)((ku0 + ku) * 32 * 2) : 0x7fff0000u;
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(e < 4 ? rx : rw,
                                             (__attribute__((address_space(3))) void*)dst, 16,
                                             voff[e], kb, 0, 0);
#endif
  };
  // ---- fragment reads: set f (0/1) of unit u: A rows wm*128 + 16 i + fr, W rows wn*128 + ...
  bf16x8 fa[2][8], fb[2][8];
  const int ra = wm * 128 + fr, rb = wn * 128 + fr;
  auto rd = [&](auto fc, int u) {
    constexpr int f = decltype(fc)::value;
    const bf16x8* slot = lds + (u & 3) * PU_SLOT;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = ra + 16 * i;
      fa[f][i] = slot[r * 4 + pu_swz(r, fg)];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = rb + 16 * j;
      fb[f][j] = slot[PG_T * 4 + r * 4 + pu_swz(r, fg)];
    }
  };
  auto mma = [&](auto fc) {
    constexpr int f = decltype(fc)::value;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[f][j], fa[f][i], acc[i][j], 0, 0, 0);
  };
  using F0 = HalfTile<0>;
  using F1 = HalfTile<1>;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: units 0..3 requested, unit 0's fragments in set 0 ----
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) dma(u, e);
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  rd(F0{}, 0);

  // one unit: wait for unit u + 1, barrier, MFMAs of u (set F) + DMA of u + 4 + reads of
  // u + 1.  ONE loop over all units, two per iteration (the register sets alternate); the
  // waits near the end are picked by uniform branches (a peeled tail made the register
  // allocator rotate the 256 accumulators through copies every iteration)
  auto step = [&](auto fc, auto gc, int u) {
    // units u + 2, u + 3 are younger than u + 1 (16 pieces).  Near the end those are dropped
    // pieces, and the waits are taken by uniform branches anyway: with one branch-free body
    // the register allocator rotated the 256 accumulators through AGPR copies every unit
    const int younger = min(nu - 2 - u, 2);
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int e = 0; e < 8; ++e) dma(u + 4, e);
    // the fragment reads of unit u + 1 (past the last unit: a harmless re-read of a landed
    // slot) and the 64 MFMAs of unit u in one scheduling region: the machine scheduler spreads
    // the DMA pieces and reads between the MFMAs itself (explicit interleaving -- per-group
    // sched_barrier fences or sched_group_barrier -- also made the allocator rotate them)
    rd(gc, u + 1);
    mma(fc);
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int u = 0; u < nu; u += 2) {  // nu even
    step(F0{}, F1{}, u);
    step(F1{}, F0{}, u + 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the main loop
}

template <int EPI, bool GROUPED, int NB, int WAVES, int SCHED = 1>
__global__ __launch_bounds__(WAVES * 64, 1) void pgemm_kernel(PGemmArgs p) {
  using G = PgGeo<WAVES>;
  constexpr int NJ = G::NJ;
  __shared__ bf16x8 lds[2 * PG_BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / G::WN, wn = w % G::WN;
  const int fr = lane & 15, fg = lane >> 4;

  // ---- tile of this workgroup --------------------------------------------------------------
  int tm, tn, group, row_lo, row_hi;
  if (!pg_tile<GROUPED>(p, tm, tn, group, row_lo, row_hi)) return;  // surplus WG (uniform)
  const int m0 = row_lo + tm * PG_T, n0 = tn * PG_T;
  const bf16* X = static_cast<const bf16*>(p.X);
  const bf16* W = static_cast<const bf16*>(p.W) + (GROUPED ? (size_t)group * p.N * p.K : 0);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)X, (short)0, (int)((size_t)p.M * p.ldx * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)W, (short)0, (int)((size_t)p.N * p.K * 2), 0x00020000);
  PgAcc<2 * PgGeo<WAVES>::NJ> accs;
  auto& acc = accs.v;
  if constexpr (SCHED == 3) {
    static_assert(WAVES == 4, "the unit-pipelined body is the 4-wave 128 x 128 form");
    const int nu = p.K / 32;
    const int id = (int)blockIdx.x;  // decorrelate ids that share an X panel (id, id + 8) and
    const int h = (id ^ (id >> 3)) & 7;  // those that share a W panel (consecutive ids)
    const int st0 = p.stagger ? (h * nu) / 8 : 0;
    pg_mainloop_u<EPI == EPI_SILU>(lds, rx, rw, p.ldx, p.K, p.N >> 1, m0, n0, 0, nu, st0,
                                   accs);
  } else {
    pg_mainloop<NB, EPI == EPI_SILU, WAVES, decltype(accs), SCHED>(lds, rx, rw, p.ldx, p.K,
                                                                   p.N >> 1, m0, n0, 0,
                                                                   p.K / PG_BK, accs);
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
      for (int jj = 0; jj < NJ; ++jj) {
        const int col = (n0 >> 1) + wn * (G::WCOLS / 2) + jj * 16 + fg * 4;
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
      for (int j = 0; j < 2 * NJ; ++j) {
        const int col = n0 + wn * G::WCOLS + j * 16 + fg * 4;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r]);
        *reinterpret_cast<bf16x4*>(Y + (size_t)row * p.ldy + col) = o;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Decode-sized M (<= a few row tiles) with the K range split over workgroups and the slices
// combined INSIDE the launch (DGemmArgs form, the decode chain's epilogues).  At M = 256 a
// Llama-3-8B projection has only N / 256 = 16 .. 112 output tiles, so one tile per workgroup
// leaves most of the 256 CUs idle; here tile t runs as `splits` workgroups, slice s taking K
// tiles [s nk / splits, (s+1) nk / splits) through the same 256 x 256 main loop, and then:
//   publish  the fp32 partial tile goes to its slab with write-through (sc1) 16-B stores, every
//            wave drains (`s_waitcnt vmcnt(0)`), the workgroup barrier, one agent-scope ticket
//            add on the tile's arrival counter (MI355X_MICROARCH.md "Valid forms", the first
//            row of the sc1 table: no release fence, no acquire);
//   combine  every slice waits (one lane, relaxed agent polls, bounded) until all `splits`
//            slices arrived -- the grid is sized <= the CU count at one 512-thread, 128 KB-LDS
//            workgroup per CU, so all slices are resident -- then reduces ITS 256 / splits
//            rows of the tile over all slabs with sc1 16-B loads and applies the epilogue
//            (row scale by ss_in, plain store / residual + next-norm / SwiGLU);
//   re-arm   the last slice to finish its rows zeroes the tile's two counters.
// The distributed combine keeps each workgroup's slab reads to 256 KB whatever the split
// (a last-arriver combine would read (splits - 1) x 256 KB on one CU).
__device__ __forceinline__ bool pg_spin_ge(const int* c, int v) {
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < v) {
    if (wall_clock64() - t0 > 100000000ull) return false;  // ~1 s: give up (error flag)
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

constexpr int kPgSc1 = 16;  // buffer op cache bits: sc1 (write-through stores, L1-bypass loads)

// sum over the `splits` slabs of the f32x4 at byte offset off (slab stride bytes): the sc1
// loads are issued 8 at a time (each is a round trip past the per-XCD L2, ~1 us; a plain loop
// over the slices would wait for every one in turn)
__device__ __forceinline__ f32x4 pg_sum_slabs(__amdgpu_buffer_rsrc_t rs, size_t off,
                                              size_t stride, int splits) {
  f32x4 y = {0.f, 0.f, 0.f, 0.f};
  for (int q0 = 0; q0 < splits; q0 += 8) {
    f32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           rs, (int)(off + min(q0 + j, splits - 1) * stride), 0,
                                           kPgSc1));
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (q0 + j < splits) y += v[j];
  }
  return y;
}

// Epilogue of 4 consecutive output columns (col) of one row, values y (fp32, before the row
// scale): EPI_STORE / EPI_RESNORM; returns the row's sum-of-squares contribution (RESNORM).
template <int EPI>
__device__ __forceinline__ float pg_epi4(const DGemmArgs& p, int row, int col, f32x4 y,
                                         float scale) {
  bf16* Y = static_cast<bf16*>(p.Y);
  bf16x4 o;
  if constexpr (EPI == EPI_RESNORM) {
    const bf16x4 r = *reinterpret_cast<const bf16x4*>(Y + (size_t)row * p.ldy + col);
    const bf16x4 g = *reinterpret_cast<const bf16x4*>(static_cast<const bf16*>(p.ln_out) + col);
    bf16x4 a;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[k] = f2bf(bf2f(f2bf(y[k] * scale)) + bf2f(r[k]));
      const float f = bf2f(o[k]);
      a[k] = f2bf(f * bf2f(g[k]));
      q += f * f;
    }
    *reinterpret_cast<bf16x4*>(Y + (size_t)row * p.ldy + col) = o;
    *reinterpret_cast<bf16x4*>(static_cast<bf16*>(p.Aout) + (size_t)row * p.N + col) = a;
    return q;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = f2bf(y[k] * scale);
    *reinterpret_cast<bf16x4*>(Y + (size_t)row * p.ldy + col) = o;
    return 0.f;
  }
}

// SwiGLU epilogue of 4 output features: gate g, up u (fp32, before the row scale)
__device__ __forceinline__ void pg_epi_silu(const DGemmArgs& p, int row, int col, f32x4 g,
                                            f32x4 u, float scale) {
  bf16x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float gg = bf2f(f2bf(g[k] * scale));
    const float uu = bf2f(f2bf(u[k] * scale));
    o[k] = f2bf(bf2f(f2bf(gg / (1.f + __expf(-gg)))) * uu);
  }
  *reinterpret_cast<bf16x4*>(static_cast<bf16*>(p.Y) + (size_t)row * p.ldy + col) = o;
}

__device__ __forceinline__ float pg_row_scale(const DGemmArgs& p, int row) {
  return p.ss_in != nullptr ? rsqrtf(p.ss_in[row] / (float)p.K + p.eps) : 1.f;
}

template <int EPI, int NB, int WAVES, int SCHED = 1>
__global__ __launch_bounds__(WAVES * 64, 1) void pgemm_sk_kernel(DGemmArgs p, int splits) {
  using G = PgGeo<WAVES>;
  constexpr int NJ = G::NJ, THREADS = G::THREADS;
  __shared__ bf16x8 lds[2 * PG_BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / G::WN, wn = w % G::WN;
  const int fr = lane & 15, fg = lane >> 4;
  const int tiles_n = p.N / PG_T;
  const int tiles_m = (p.M + PG_T - 1) / PG_T;
  const int nwg = tiles_m * tiles_n * splits;
  const int id = xcd_remap(blockIdx.x, nwg);  // a tile's slices on consecutive ids (one XCD)
  const int tile = id / splits, s = id % splits;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * PG_T, n0 = tn * PG_T;
  const int nk = p.K / PG_BK;
  const int kt0 = s * nk / splits, kt1 = (s + 1) * nk / splits;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.X), (short)0, (int)((size_t)p.M * p.ldx * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.W), (short)0, (int)((size_t)p.N * p.ldw * 2), 0x00020000);
  PgAcc<2 * PgGeo<WAVES>::NJ> accs;
  auto& acc = accs.v;
  pg_mainloop<NB, EPI == EPI_SILU, WAVES, decltype(accs), SCHED>(lds, rx, rw, p.ldx, p.ldw,
                                                                 p.N >> 1, m0, n0, kt0,
                                                                 kt1 - kt0, accs);

  if (splits == 1) {  // whole K in this workgroup: the epilogue straight from the registers
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = m0 + wm * 128 + i * 16 + fr;
      if (row >= p.M) continue;
      const float sc = pg_row_scale(p, row);
      if constexpr (EPI == EPI_SILU) {
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj)
          pg_epi_silu(p, row, (n0 >> 1) + wn * (G::WCOLS / 2) + jj * 16 + fg * 4,
                      acc[i][2 * jj], acc[i][2 * jj + 1], sc);
      } else {
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 2 * NJ; ++j)
          q += pg_epi4<EPI>(p, row, n0 + wn * G::WCOLS + j * 16 + fg * 4, acc[i][j], sc);
        if constexpr (EPI == EPI_RESNORM) atomicAdd(p.ss_out + row, q);
      }
    }
    return;
  }
  // ---- publish the partial tile (write-through), take a ticket ----
  constexpr int SLAB = PG_T * PG_T;  // floats
  float* slabs = p.ws + (size_t)tile * splits * SLAB;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)slabs, (short)0, (int)((size_t)splits * SLAB * 4), 0x00020000);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2 * NJ; ++j) {
      const int r = wm * 128 + i * 16 + fr, c = wn * G::WCOLS + j * 16 + fg * 4;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                             (int)(((size_t)s * SLAB + r * PG_T + c) * 4), 0,
                                             kPgSc1);
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its stores
  __syncthreads();
  int* arrive = p.counters + 2 * tile * kCtrStride;  // arrivals (polled) and finishes: each
  int* done = arrive + kCtrStride;                     // on its own L2 line
  if (tid == 0) {
    __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!pg_spin_ge(arrive, splits))
      __hip_atomic_fetch_or(p.counters + kCtrErr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  // ---- combine rows [r0, r1) of the tile over every slab (sc1 loads) ----
  const int r0 = s * PG_T / splits, r1 = (s + 1) * PG_T / splits;
  if constexpr (EPI == EPI_SILU) {
    // a row has 32 gate chunks of 4 columns; gate chunk cg <-> tile columns 32 (cg/4) + 4 (cg%4)
    // (gate) and + 16 (up): output features n0/2 + 16 (cg/4) + 4 (cg%4) .. + 3
    for (int e = tid; e < (r1 - r0) * 32; e += THREADS) {
      const int r = r0 + e / 32, cg = e % 32;
      const int row = m0 + r;
      if (row >= p.M) continue;
      const int cgate = (cg >> 2) * 32 + (cg & 3) * 4;
      const size_t base = ((size_t)r * PG_T + cgate) * 4;
      const f32x4 g = pg_sum_slabs(rs, base, (size_t)SLAB * 4, splits);
      const f32x4 u = pg_sum_slabs(rs, base + 64, (size_t)SLAB * 4, splits);
      pg_epi_silu(p, row, (n0 >> 1) + (cg >> 2) * 16 + (cg & 3) * 4, g, u, pg_row_scale(p, row));
    }
  } else {
    // 64 chunks of 4 columns per row; with RESNORM the 64 lanes of a wave own one row (its
    // sum of squares is reduced across the wave, one atomic per row)
    for (int e = tid; e < (r1 - r0) * 64; e += THREADS) {
      const int r = r0 + e / 64, c = (e % 64) * 4;
      const int row = m0 + r;
      const f32x4 y = pg_sum_slabs(rs, ((size_t)r * PG_T + c) * 4, (size_t)SLAB * 4, splits);
      float qs = 0.f;
      if (row < p.M) qs = pg_epi4<EPI>(p, row, n0 + c, y, pg_row_scale(p, row));
      if constexpr (EPI == EPI_RESNORM) {
        qs = wave_sum(qs);
        if (lane == 0 && row < p.M) atomicAdd(p.ss_out + row, qs);
      }
    }
  }
  // ---- re-arm the tile's counters (the last slice to finish its rows) ----
  __syncthreads();
  if (tid == 0) {
    const int d = __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == splits - 1) {
      __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

bool pgemm_sk_supported(int M, int N, int K, int splits, int cus) {
  const int nk = K / PG_BK;
  const long grid = (long)((M + PG_T - 1) / PG_T) * (N / PG_T) * splits;
  return M > 0 && N % PG_T == 0 && K % PG_BK == 0 && splits >= 1 && splits <= 32 &&
         nk >= splits && grid <= cus &&
         (N / PG_T) * ((M + PG_T - 1) / PG_T) * 2 * kCtrStride < kCtrErr;
}

long pgemm_sk_ws_floats(int M, int N, int splits) {
  if (splits <= 1) return 0;
  return (long)((M + PG_T - 1) / PG_T) * (N / PG_T) * splits * PG_T * PG_T;
}

// Wave form of the 256 x 256 body: AKAP_PGEMM_WAVES = 8 (2 x 4 waves of 128 x 64) or 4 (2 x 2
// waves of 128 x 128), read once per process.
// K-loop issue schedule: AKAP_PGEMM_SCHED = 1 (phase pipeline, half-tiles requested 1.0-1.25
// tiles ahead), 2 (early issue, 1.25-1.75 tiles ahead), 3 (4-wave unit body), 4 (default,
// stream-first: the whole next tile under this tile's math, 5-14 % faster than 1 on the dense
// verdict shapes, profiles/r6_pgemm_isa_diff.md; pg_mainloop), read once per process.  The
// decode split-K form (launch_pgemm_sk) keeps 1 / 2.
int pgemm_sched() {
  static int v = [] {
    const char* e = getenv("AKAP_PGEMM_SCHED");
    const int x = e ? atoi(e) : 4;  // default: the stream-first body (r6_pgemm_isa_diff.md)
    return (x >= 1 && x <= 4) ? x : 4;
  }();
  return v;
}

int pgemm_waves() {
  static int w = [] {
    const char* e = getenv("AKAP_PGEMM_WAVES");
    return (e && atoi(e) == 4) ? 4 : 8;
  }();
  return w;
}

template <int WAVES, int SCHED>
static void launch_pgemm_sk_w(const DGemmArgs& p, int splits, hipStream_t st) {
  const int grid = ((p.M + PG_T - 1) / PG_T) * (p.N / PG_T) * splits;
  constexpr int T = WAVES * 64;
  if (p.epi == EPI_SILU)
    pgemm_sk_kernel<EPI_SILU, 4, WAVES, SCHED><<<grid, T, 0, st>>>(p, splits);
  else if (p.epi == EPI_RESNORM)
    pgemm_sk_kernel<EPI_RESNORM, 2, WAVES, SCHED><<<grid, T, 0, st>>>(p, splits);
  else pgemm_sk_kernel<EPI_STORE, 2, WAVES, SCHED><<<grid, T, 0, st>>>(p, splits);
}

void launch_pgemm_sk(const DGemmArgs& p, int splits, hipStream_t st) {
  if (p.M == 0) return;
  if (pgemm_waves() == 4) {  // (SCHED 3 / 4 are whole-tile bodies: the split-K form runs 1)
    if (pgemm_sched() == 2) launch_pgemm_sk_w<4, 2>(p, splits, st);
    else launch_pgemm_sk_w<4, 1>(p, splits, st);
  } else {
    if (pgemm_sched() == 2) launch_pgemm_sk_w<8, 2>(p, splits, st);
    else launch_pgemm_sk_w<8, 1>(p, splits, st);
  }
}

bool pgemm_supported(int M, int N, int K) {
  return M > 0 && N > 0 && N % PG_T == 0 && K >= PG_BK && K % PG_BK == 0;
}

template <int WAVES, int SCHED>
static void launch_pgemm_w(const PGemmArgs& p, int epi, int grid, hipStream_t st) {
  constexpr int T = WAVES * 64;
  if (p.groups > 0) {
    if (epi == EPI_SILU) pgemm_kernel<EPI_SILU, true, 4, WAVES, SCHED><<<grid, T, 0, st>>>(p);
    else pgemm_kernel<EPI_STORE, true, 2, WAVES, SCHED><<<grid, T, 0, st>>>(p);
  } else {
    if (epi == EPI_SILU) pgemm_kernel<EPI_SILU, false, 4, WAVES, SCHED><<<grid, T, 0, st>>>(p);
    else pgemm_kernel<EPI_STORE, false, 2, WAVES, SCHED><<<grid, T, 0, st>>>(p);
  }
}

void launch_pgemm(const PGemmArgs& a, int epi, hipStream_t st) {
  if (a.M == 0) return;
  static const int gm = [] {  // raster block height (AKAP_PGEMM_GM, A/B knob; default 8)
    const char* e = getenv("AKAP_PGEMM_GM");
    return e ? atoi(e) : 0;
  }();
  PGemmArgs p = a;
  p.gm = gm;
  const int tiles_n = p.N / PG_T;
  const int grid = p.groups > 0 ? ((p.M + PG_T - 1) / PG_T + p.groups) * tiles_n
                                 : ((p.M + PG_T - 1) / PG_T) * tiles_n;
  if (pgemm_sched() == 3 && p.K % 128 == 0) {  // unit-pipelined 4-wave body (K >= 128)
    static const int stag = [] {
      const char* e = getenv("AKAP_PGEMM_STAGGER");
      return e ? atoi(e) : 0;
    }();
    PGemmArgs q = p;
    q.stagger = stag;
    launch_pgemm_w<4, 3>(q, epi, grid, st);
    return;
  }
  if (pgemm_sched() == 4) {  // stream-first body (AKAP_PGEMM_WAVES 8 | 4)
    if (pgemm_waves() == 4) launch_pgemm_w<4, 4>(p, epi, grid, st);
    else launch_pgemm_w<8, 4>(p, epi, grid, st);
    return;
  }
  // two barriers per K tile (measured 1-4 % faster than four, profiles/r4_pgemm_nb_ab.log); the
  // SwiGLU form keeps four: with both fragment sets read in phase 1 it would spill
  const bool s2 = pgemm_sched() == 2;
  if (pgemm_waves() == 4) {
    if (s2) launch_pgemm_w<4, 2>(p, epi, grid, st);
    else launch_pgemm_w<4, 1>(p, epi, grid, st);
  } else {
    if (s2) launch_pgemm_w<8, 2>(p, epi, grid, st);
    else launch_pgemm_w<8, 1>(p, epi, grid, st);
  }
}

}  // namespace akap
