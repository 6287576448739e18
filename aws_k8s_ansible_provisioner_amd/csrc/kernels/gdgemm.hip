// Decode GEMM with LDS-DMA operand staging for gfx950:  Y[M,N] = X[M,K] . W[N,K]^T
// (plain prologue + the dgemm.hip epilogues: store / residual+next-norm / SwiGLU, optional
// ss_in row scale).
//
// Why: at decode sizes (M <= 256) these GEMMs are latency bound -- every block walks its K
// range as a chain of HBM/L2 round trips, and a CU only streams as fast as the bytes it
// keeps in flight allow (in-flight bytes / load latency; MI355X_MICROARCH.md price-table rows
// ldsdma-fill / ring-gemm).  global_load_lds writes LDS directly (no VGPR round trip, no
// ds_write pass), so the ring depth is bounded by LDS, not registers:
//   shallow ring: NS = 4 (64-col) / 3 (128-col) slots, two blocks per CU;
//   deep ring:    NS = 8 (64-col, 128 KB) / 6 (128-col, 144 KB), one block per CU and
//                 NS-1 k-steps (112-120 KB) in flight -- for grids of <= 256 tiles.
//
// Structure: BM x BN output tile (BM 64 | 128 | 256, BN 64 | 128), BK = 64; 4 waves as 2 (M)
// x 2 (N), or for BM = 256 8 waves as 4 (M) x 2 (N) (512 threads, wave tile 64 x BN/2).
// BM = 128 (wave tile 64 x 64) halves the weight traffic of a 256-row batch (each weight byte
// crosses L2 -> CU twice instead of four times): the large-weight projections of Llama-3-8B
// class models, where the decode GEMMs are weight-stream bound.  BM = 256 covers the whole
// 256-row batch: every weight byte crosses L2 -> CU exactly once and each CU's load path
// carries (256 + BN) rows per k-step for 256 x BN outputs -- 85 FLOP per staged byte at
// BN = 128 (vs 64 for 128 x 128) -- so the 8B / 70B-shard projections at M = 256, which sit
// at the MFMA / L2-bandwidth ridge, stream their weights once at up to the MFMA rate.  Per
// k-step: counted `s_waitcnt vmcnt` for this step's DMAs, raw s_barrier (never
// __syncthreads: its fence would drain every DMA in flight), refill the slot consumed one step
// earlier, then ds_read fragments + MFMA 16x16x32.  LDS image: linear DMA destination, XOR
// swizzle applied to the per-lane SOURCE address and to the fragment reads (the same
// involution, cdna_hip_programming.md rule 21).
//
// Split-K (gridDim.y = S slices):
//   SPL 1: fp32 partial slabs [S, M, N], reduced (with the epilogue) by dgemm.hip's reduce pass;
//   SPL 2: in-launch combine.  Every slice stores its accumulators as a fragment-native slab
//          (16 B per lane per MFMA tile, fully coalesced) with write-through (sc1) stores, every
//          wave drains (`s_waitcnt vmcnt(0)`), the workgroup barrier, then lane 0 takes an
//          agent-scope ticket on the tile's counter (its own L2 line, kCtrStride) -- the sc1
//          hand-off of MI355X_MICROARCH.md "Valid forms" (no release / acquire fence: each
//          costs ~1.7 us and more behind a dirty L2).  The slice that draws S-1 re-arms the
//          ticket and sums the S slabs with sc1 loads, then runs the epilogue.  No second
//          launch, so the GEMM -> reduce kernel boundary (~1.5 us) and the reduce body go away,
//          and split-K becomes legal for the SwiGLU epilogue too.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int GBK = 64;
constexpr int kGdSc1 = 16;  // buffer op cache bits: sc1 (write-through stores, L1-bypass loads)

__device__ __forceinline__ int gswz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }

// LDS image of a BKT-deep k-step: rows of BKT * 2 bytes in 16-B chunks, XOR-swizzled so the 16
// lanes of a ds_read_b128 lane group (16 consecutive rows, one chunk) hit 16 distinct 16-B bank
// positions.  BKT = 64: 8 chunks per row, chunk ^ (row & 7).  BKT = 32: 4 chunks per row (four
// rows per 256-B bank row), chunk ^ ((row >> 2) & 3).
template <int BKT>
__device__ __forceinline__ int gswz_t(int row, int chunk) {
  if constexpr (BKT == 64) return row * 8 + (chunk ^ (row & 7));
  else return row * 4 + (chunk ^ ((row >> 2) & 3));
}

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0,
                                   0);
}
// the same with the non-temporal policy: once-read decode weights (MI355X_MICROARCH.md
// nt-weights), never for the activation rows every column tile re-reads
__device__ __forceinline__ void glds16_nt(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0,
                                   2);
}

// AKAP_WEIGHT_NT: unset -> -1 (gdgemm weights non-temporal, kgemm default policy: measured
// Llama-3-8B +0.7 % on both A/B pairs, Qwen3-0.6B -0.65 % with kgemm nt too,
// profiles/r3_weight_nt_ab.log); 1 -> both non-temporal; 0 -> neither
int gemm_stagger_default() {
  static const int v = [] {
    const char* e = std::getenv("AKAP_GEMM_STAGGER");
    return e == nullptr ? 0 : std::atoi(e);
  }();
  return v;
}

int weight_nt_default() {
  static const int v = [] {
    const char* e = std::getenv("AKAP_WEIGHT_NT");
    return e == nullptr ? -1 : (std::atoi(e) == 1 ? 1 : 0);
  }();
  return v;
}

template <int N_>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N_ >= 63) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

// BKT: k-step depth (64 in every served variant).  Measured and removed: a 6-slot ring of
// 32-deep k-steps for the 256-row tiles (five in flight; slower on every M = 256 shape,
// profiles/r3_gemm_m256_deep.log) and a half-step pipelined K loop (fragment reads of the next
// half-step under the current MFMAs; within 2 %, profiles/r3_gemm_pipe_ab.log).
template <int BN, int NS, int EPI, int SPL, int OCC, int S, int GBM = 64, int NW = 4,
          int BKT = 64>
__global__ __launch_bounds__(64 * NW, OCC) void gdgemm_kernel(DGemmArgs p) {
  constexpr int NT = 64 * NW;             // threads
  constexpr int WMW = NW / 2;             // waves along M (2 along N)
  constexpr int WR = GBM / WMW;           // wave tile rows (wave tile WR x BN/2)
  constexpr int CPR = BKT / 8;            // 16-B chunks per staged row
  constexpr int RPI = 64 / CPR;           // rows per DMA instruction (64 lanes x 16 B)
  constexpr int SU = (GBM + BN) * CPR;    // slot size in 16-B units
  constexpr int MI = WR / 16;             // 16-row MFMA tiles per wave
  constexpr int JN = BN / 32;             // 16-col MFMA tiles per wave
  constexpr int GA = GBM / (RPI * NW), GW = BN / (RPI * NW);  // DMA instrs per wave per k-step
  constexpr int G = GA + GW;
  static_assert(BKT == 64 || BKT == 32, "k-step 64 | 32");
  static_assert(GA * RPI * NW == GBM && GW * RPI * NW == BN, "DMA pieces cover the tile");
  // ONE __shared__ object (a second one makes hipcc drain vmcnt inside the k-loop,
  // cdna_hip_programming.md "Projection GEMM at M = 256" item 4a); the last element is the
  // split-K "this block combines" flag
  __shared__ bf16x8 lds[NS * SU + 1];

  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles_m = (p.M + GBM - 1) / GBM;
  const int ntiles = tiles_n * tiles_m;
  const int lt = xcd_remap(blockIdx.x, ntiles);
  const int tn = lt / tiles_m, tm = lt % tiles_m;
  const int m0 = tm * GBM, n0 = tn * BN;
  const int kz = blockIdx.y;
  const int kbeg = kz * p.kps;
  const int nk = p.kps / BKT;
  const int st0 = gemm_stagger0(p.stag, tm, tn, nk);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const bf16* X = static_cast<const bf16*>(p.X);
  const bf16* W = static_cast<const bf16*>(p.W);
  bf16* Y = static_cast<bf16*>(p.Y);

  // per-lane DMA sources: an instruction covers RPI rows x BKT*2 B; lane -> row L/CPR, LDS
  // chunk L%CPR holding the logical chunk that gswz_t maps there (the swizzle's row bits are
  // the lane's: every instruction starts on a multiple of RPI rows)
  const int lr = lane / CPR;
  const int lc = BKT == 64 ? (lane & 7) ^ (lane >> 3) : (lane & 3) ^ ((lane >> 4) & 3);
  const bf16* asrc[GA];
  const bf16* wsrc[GW];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int row = m0 + (w * GA + i) * RPI + lr;
    asrc[i] = X + (size_t)(row < p.M ? row : 0) * p.ldx + lc * 8;
  }
#pragma unroll
  for (int i = 0; i < GW; ++i) {
    const int v = n0 + (w * GW + i) * RPI + lr;
    int wrow = v < p.N ? v : 0;
    if constexpr (EPI == EPI_SILU)
      wrow = v < p.N ? ((v >> 4) & 1) * (p.N >> 1) + (v >> 5) * 16 + (v & 15) : 0;
    wsrc[i] = W + (size_t)wrow * p.ldw + lc * 8;
  }
  auto issue = [&](int step) {  // DMA k-step `step` into its ring slot
    bf16x8* slot = lds + (step % NS) * SU;
    int ks = step + st0;
    if (ks >= nk) ks -= nk;
    const int k0 = kbeg + ks * BKT;
#pragma unroll
    for (int i = 0; i < GA; ++i) glds16(asrc[i] + k0, slot + (w * GA + i) * 64);
    if (p.ntw != 0) {
#pragma unroll
      for (int i = 0; i < GW; ++i) glds16_nt(wsrc[i] + k0, slot + GBM * CPR + (w * GW + i) * 64);
    } else {
#pragma unroll
      for (int i = 0; i < GW; ++i) glds16(wsrc[i] + k0, slot + GBM * CPR + (w * GW + i) * 64);
    }
  };

  // epilogue operands from the previous launch: load before the loop (hidden under it)
  constexpr bool EPI_HERE = SPL != 1;  // this launch runs the epilogue (no separate reduce)
  float rsc[MI][4];
  bf16 rold[MI][4][JN];
  bf16 lnv[JN];
  const float* ssp = p.ss_in != nullptr ? p.ss_in : static_cast<const float*>(p.W);
  if constexpr (EPI_HERE) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * WR + i * 16 + fg * 4 + r;
        const int rowc = row < p.M ? row : 0;
        rsc[i][r] = ssp[rowc];
        if constexpr (EPI == EPI_RESNORM) {
#pragma unroll
          for (int j = 0; j < JN; ++j) {
            const int col = n0 + wn * (BN / 2) + j * 16 + fr;
            rold[i][r][j] = Y[(size_t)rowc * p.ldy + (col < p.N ? col : 0)];
          }
        }
      }
    if constexpr (EPI == EPI_RESNORM) {
      const bf16* lno = static_cast<const bf16*>(p.ln_out);
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        const int col = n0 + wn * (BN / 2) + j * 16 + fr;
        lnv[j] = lno[col < p.N ? col : 0];
      }
    }
  }

  f32x4 acc[MI][JN];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: up to NS-1 k-steps in flight.  At step t the wait below leaves the NS-2 later
  // steps in flight only when all of them exist (t + NS - 2 < nk), else drains to 0, so a
  // short K range (nk < NS - 1) is handled by the same counts.
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s);
  for (int t = 0; t < nk; ++t) {
    // retire this thread's DMAs of step t: the later steps issued so far stay in flight
    if (t + NS - 2 < nk) wait_vm<G * (NS - 2)>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMAs of step t landed; slot t-1 is free
    if (t + NS - 1 < nk) issue(t + NS - 1);
    const bf16x8* slot = lds + (t % NS) * SU;
#pragma unroll
    for (int ks = 0; ks < BKT / 32; ++ks) {
      bf16x8 af[MI], bfr[JN];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = slot[gswz_t<BKT>(wm * WR + i * 16 + fr, ks * 4 + fg)];
#pragma unroll
      for (int j = 0; j < JN; ++j)
        bfr[j] = slot[GBM * CPR + gswz_t<BKT>(wn * (BN / 2) + j * 16 + fr, ks * 4 + fg)];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  if constexpr (SPL == 2) {
    // ---- in-launch split-K combine (see header) ----
    constexpr int NF = MI * JN;  // f32x4 fragments per lane
    const size_t tile_stride = (size_t)NF * NT;
    const size_t zs = (size_t)ntiles * tile_stride;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        p.ws, (short)0, (int)((size_t)S * zs * 16), 0x00020000);
    const size_t mine = ((size_t)kz * ntiles + lt) * tile_stride + tid;  // f32x4 units
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                               (int)((mine + (size_t)(i * JN + j) * NT) * 16), 0,
                                               kGdSc1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its stores
    __syncthreads();
    int* flag = reinterpret_cast<int*>(&lds[NS * SU]);
    int* ticket = p.counters + (size_t)lt * kCtrStride;
    if (tid == 0) {
      const int prev = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == S - 1;
      if (last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (*flag == 0) return;
    // the combining block sums all S slabs (its own included: one code path, every load
    // issued back to back -- no per-slice runtime condition around a load); sc1 loads miss
    // the (per-XCD, non-coherent) caches a slice on another XCD could not have written through
    const size_t t0 = (size_t)lt * tile_stride + tid;
#pragma unroll
    for (int f = 0; f < NF; ++f)
      acc[f / JN][f % JN] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((t0 + f * NT) * 16), 0, kGdSc1));
    // every slice's fragments (NF per slab) requested before any is summed: one round trip
    // past the per-XCD L2 per slab, overlapped
    for (int z = 1; z < S; ++z) {
      f32x4 v[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f)
        v[f] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((t0 + z * zs + f * NT) * 16),
                                                         0, kGdSc1));
#pragma unroll
      for (int f = 0; f < NF; ++f) acc[f / JN][f % JN] += v[f];
    }
  }

  // epilogue: lane holds rows wm*WR + i*16 + fg*4 + r, column fr of each 16-col sub-tile
  const float inv_k = 1.f / (float)p.K;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm * WR + i * 16 + fg * 4 + r;
      const bool row_ok = row < p.M;
      if constexpr (SPL == 1) {
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int col = n0 + wn * (BN / 2) + j * 16 + fr;
          if (row_ok && col < p.N) p.ws[((size_t)kz * p.M + row) * p.N + col] = acc[i][j][r];
        }
        continue;
      }
      float scale = 1.f;
      if (p.ss_in != nullptr) scale = rsqrtf(rsc[i][r] * inv_k + p.eps);
      if constexpr (EPI == EPI_STORE) {
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int col = n0 + wn * (BN / 2) + j * 16 + fr;
          if (row_ok && col < p.N) Y[(size_t)row * p.ldy + col] = f2bf(acc[i][j][r] * scale);
        }
      } else if constexpr (EPI == EPI_RESNORM) {
        bf16* Ao = static_cast<bf16*>(p.Aout);
        float q2 = 0.f;
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int col = n0 + wn * (BN / 2) + j * 16 + fr;
          if (row_ok && col < p.N) {
            const bf16 s = f2bf(bf2f(f2bf(acc[i][j][r] * scale)) + bf2f(rold[i][r][j]));
            Y[(size_t)row * p.ldy + col] = s;
            const float f = bf2f(s);
            Ao[(size_t)row * p.N + col] = f2bf(f * bf2f(lnv[j]));
            q2 += f * f;
          }
        }
        q2 += __shfl_xor(q2, 1, kWave);
        q2 += __shfl_xor(q2, 2, kWave);
        q2 += __shfl_xor(q2, 4, kWave);
        q2 += __shfl_xor(q2, 8, kWave);
        if (fr == 0 && row_ok) atomicAdd(p.ss_out + row, q2);
      } else {  // EPI_SILU: sub-tiles 2jj / 2jj+1 = gate / up of one 16-feature group
#pragma unroll
        for (int jj = 0; jj < JN / 2; ++jj) {
          const int vb = n0 + wn * (BN / 2) + 32 * jj;
          if (row_ok && vb + 16 + fr < p.N) {
            const float g = bf2f(f2bf(acc[i][2 * jj][r] * scale));
            const float u = bf2f(f2bf(acc[i][2 * jj + 1][r] * scale));
            const float sg = bf2f(f2bf(g / (1.f + __expf(-g))));
            Y[(size_t)row * p.ldy + (vb >> 1) + fr] = f2bf(sg * u);
          }
        }
      }
    }
}

bool gdgemm_supported(int M, int N, int K, int splitk, int bn, int bm) {
  if (bn != 64 && bn != 128) return false;
  if (bm != 64 && !(bm == 128 && bn == 128) && bm != 256) return false;
  if (M <= 0 || N <= 0 || K <= 0 || !dgemm_splitk_ok(splitk) || N % 4 || K % splitk) return false;
  const int kps = K / splitk;
  return kps % GBK == 0 && kps >= GBK;
}

long gdgemm_ws_floats(int M, int N, int splitk, int bn, int bm) {
  const long tm = (M + bm - 1) / bm, tn = (N + bn - 1) / bn;
  const long slabs = (long)splitk * tm * tn * bm * bn;
  const long dense = (long)splitk * M * N;
  return slabs > dense ? slabs : dense;
}

template <int BN, int NS, int OCC, int SPL, int S, int BM, int NW>
static void gdgemm_epi(const DGemmArgs& p, dim3 grid, hipStream_t st) {
  if (p.epi == EPI_RESNORM) {
    gdgemm_kernel<BN, NS, EPI_RESNORM, SPL, OCC, S, BM, NW>
        <<<grid, 64 * NW, 0, st>>>(p);
  } else if (p.epi == EPI_SILU) {
    if constexpr (SPL != 1)
      gdgemm_kernel<BN, NS, EPI_SILU, SPL, OCC, S, BM, NW>
          <<<grid, 64 * NW, 0, st>>>(p);
  } else {
    gdgemm_kernel<BN, NS, EPI_STORE, SPL, OCC, S, BM, NW>
        <<<grid, 64 * NW, 0, st>>>(p);
  }
}

template <int BN, int NS, int OCC, int BM = 64, int NW = 4>
static void gdgemm_ring(const DGemmArgs& p, dim3 grid, int splitk, hipStream_t st) {
  if (splitk == 1) {
    gdgemm_epi<BN, NS, OCC, 0, 1, BM, NW>(p, grid, st);
  } else if (p.counters == nullptr) {
    gdgemm_epi<BN, NS, OCC, 1, 1, BM, NW>(p, grid, st);
    launch_dgemm_reduce(p, PRO_PLAIN, splitk, st);
  } else {
    switch (splitk) {
      case 2: gdgemm_epi<BN, NS, OCC, 2, 2, BM, NW>(p, grid, st); break;
      case 4: gdgemm_epi<BN, NS, OCC, 2, 4, BM, NW>(p, grid, st); break;
      case 8: gdgemm_epi<BN, NS, OCC, 2, 8, BM, NW>(p, grid, st); break;
      default:  // 16 slices: slabs + the separate reduce pass
        gdgemm_epi<BN, NS, OCC, 1, 1, BM, NW>(p, grid, st);
        launch_dgemm_reduce(p, PRO_PLAIN, splitk, st);
        break;
    }
  }
}

void launch_gdgemm(const DGemmArgs& p, int splitk, hipStream_t st) {
  const int bm = (p.bm == 128 || p.bm == 256) ? p.bm : 64;
  const int tiles = ((p.M + bm - 1) / bm) * ((p.N + p.bn - 1) / p.bn);
  dim3 grid(tiles, splitk);
  const bool deep = p.ns >= 6;
  if (bm == 256) {  // 256-row tiles, 8 waves: 3 x 48 KB (BN 128) / 3 x 40 KB (BN 64) ring
    if (p.bn == 128) gdgemm_ring<128, 3, 1, 256, 8>(p, grid, splitk, st);
    else gdgemm_ring<64, 3, 1, 256, 8>(p, grid, splitk, st);
    return;
  }
  if (bm == 128) {  // 128 x 128 tiles: 4 x 32 KB ring, one block per CU
    gdgemm_ring<128, 4, 1, 128>(p, grid, splitk, st);
    return;
  }
  // shallow: NS = 4 (64-col: 4 x 16 KB) / 3 (128-col: 3 x 24 KB) -> two blocks per CU;
  // deep: 8 x 16 KB / 6 x 24 KB -> one block per CU
  if (p.bn == 128) {
    if (deep) gdgemm_ring<128, 6, 1>(p, grid, splitk, st);
    else gdgemm_ring<128, 3, 2>(p, grid, splitk, st);
  } else {
    if (deep) gdgemm_ring<64, 8, 1>(p, grid, splitk, st);
    else gdgemm_ring<64, 4, 2>(p, grid, splitk, st);
  }
}

}  // namespace akap
