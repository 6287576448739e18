// Fused decode GEMM for gfx950:  Y[M,N] = A[M,K] . W[N,K]^T  with the elementwise work of a
// decode layer folded into the GEMMs, so a layer needs no separate RMSNorm / SwiGLU launch
// (each costs a ~1.5 us kernel boundary + a 5-6 us latency-bound body at M <= 256,
// MI355X_MICROARCH.md price table "boundary").
//
// Prologues (applied while staging A):
//   PRO_PLAIN   A = X; if ss_in is given, Y rows are scaled by rsqrt(ss_in[m] / K + eps)
//               -- the RMSNorm's per-row scale commutes with the GEMM, so a producer that
//               wrote A = bf16(s * ln) and sum_k s^2 (EPI_RESNORM below) leaves the consumer
//               a plain GEMM with a scaled epilogue: no per-N-tile recomputation of the norm.
//   PRO_ADDNORM s = bf16(X + R) (written to Rout by the n-tile-0 blocks), A = bf16(s * ln[k]),
//               Y = rsqrt(mean_k(s^2) + eps) * (A . W^T) (sum of squares from the A rows the
//               block streams anyway; split-K: per-slice partial sums, combined by the reduce)
//   PRO_SILU    X = [G | U] ([M, 2K]),  A = bf16(bf16(silu(G)) * U)
//   ADDNORM / SILU redo the elementwise op in every N-tile block (N/64-fold VALU work:
//   ~6 us at M=256 on Qwen3-0.6B shapes, profiles/r1_dgemm_micro.log); the epilogue forms
//   below do it once per output element instead and are what the engine uses.
// Epilogues:
//   EPI_STORE   Y = bf16(acc)
//   EPI_RESNORM Y is the residual stream (in/out): s = bf16(bf16(acc) + Y);  Y = s;
//               Aout = bf16(s * ln_out[n]);  ss_out[m] += sum_n s^2 (fp32 atomics, caller
//               zeroes ss_out) -- the residual add and the next RMSNorm's elementwise half.
//   EPI_SILU    W rows are read gate/up-interleaved in 16-row groups (virtual column v ->
//               weight row ((v>>4)&1) * N/2 + (v>>5) * 16 + (v&15)), so a lane's two 16-col
//               MFMA tiles hold gate and up of the same feature:
//               Y[m, f] = bf16(bf16(silu(g)) * u), Y is [M, N/2].  No weight re-layout.
//
// Geometry: 64x64 output tile, 4 waves as 2x2 each owning a 32x32 sub-tile (2x2
// v_mfma_f32_16x16x32_bf16), BK = 64, XOR-swizzled LDS double buffer, XCD-aware tile order,
// split-K over gridDim.y.  The load pipeline keeps PF k-tiles of global loads in flight in
// registers (a compile-time ring, loop unrolled by PF so every register index is static and
// the compiler's vmcnt counting stays exact), because at decode sizes each block's K loop is
// a chain of HBM/L2 round trips, not math.
#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int DBM = 64, DBN = 64, DBK = 64;
constexpr int kDgSc1 = 16;  // buffer op cache bits: sc1 (write-through stores, L1-bypass loads)

__device__ __forceinline__ int dswz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }

__device__ __forceinline__ float silu_bf(float g) { return bf2f(f2bf(g / (1.f + __expf(-g)))); }

// SPL: 0 whole K, 1 fp32 partial slabs for the separate reduce pass, 2 in-launch combine of
// the S slices (plain prologue only): fragment-native sc1 slabs + a per-tile last-arriver ticket,
// as gdgemm.hip SPL 2 -- the reduce launch (5.0 us at Qwen3 down, M = 256) and its kernel
// boundary go away (VERDICT r5 "Step A")
template <int PRO, int EPI, int PF, int SPL, int S = 1>
__global__ __launch_bounds__(256, 2) void dgemm_kernel(DGemmArgs p) {
  static_assert(SPL != 2 || PRO == PRO_PLAIN, "in-launch combine: plain prologue");
  // ONE __shared__ object (a second one makes hipcc drain vmcnt inside the k-loop,
  // cdna_hip_programming.md "Projection GEMM at M = 256" item 4a):
  // [buf 2][A|B][64 rows * 8 chunks] bf16x8, then 64 fp32 row sums of squares
  __shared__ bf16x8 lds[2 * 2 * DBM * 8 + 16];
  float* rowss = reinterpret_cast<float*>(&lds[2 * 2 * DBM * 8]);

  const int tiles_n = (p.N + DBN - 1) / DBN;
  const int tiles_m = (p.M + DBM - 1) / DBM;
  const int lt = xcd_remap(blockIdx.x, tiles_n * tiles_m);
  const int tn = lt / tiles_m;
  const int tm = lt % tiles_m;
  const int m0 = tm * DBM, n0 = tn * DBN;
  const int kz = blockIdx.y;
  const int kbeg = kz * p.kps;
  const int nk = p.kps / DBK;  // host: K % kps == 0, kps % (DBK * PF) == 0
  const int st0 = gemm_stagger0(p.stag, tm, tn, nk);
  auto kpos = [&](int i) {  // K offset of this workgroup's i-th k-tile (staggered walk)
    int ks = i + st0;
    if (ks >= nk) ks -= nk;
    return kbeg + ks * DBK;
  };
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int fr = lane & 15, fg = lane >> 4;  // MFMA fragment column / row group of this lane

  // staging: thread -> chunk tid%8 of rows tid/8 and tid/8 + 32 of both 64x64 tiles, so
  // each load instruction reads 8 whole 128-B lines (full-line staging:
  // cdna_hip_programming.md "Projection GEMM at M = 256" x-operand row).
  // Rows past M / N are clamped to row 0 (valid memory, results never stored).
  const int s_ch = tid & 7;
  const bf16* X = static_cast<const bf16*>(p.X);
  const bf16* W = static_cast<const bf16*>(p.W);
  const bf16* LN = static_cast<const bf16*>(p.ln);
  bf16* Y = static_cast<bf16*>(p.Y);
  int s_row[2];
  bool a_ok[2];
  const bf16* xa[2];
  const bf16* wb[2];
  const bf16* rr[2];
  bf16* ro[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    s_row[c] = (tid >> 3) + 32 * c;
    a_ok[c] = (m0 + s_row[c]) < p.M;
    const int v = n0 + s_row[c];  // virtual output column staged by this thread
    const bool b_ok = v < p.N;
    int wrow = b_ok ? v : 0;
    if constexpr (EPI == EPI_SILU)
      wrow = b_ok ? ((v >> 4) & 1) * (p.N >> 1) + (v >> 5) * 16 + (v & 15) : 0;
    const size_t arow = (size_t)(a_ok[c] ? m0 + s_row[c] : 0);
    xa[c] = X + arow * p.ldx;
    wb[c] = W + (size_t)wrow * p.ldw;
    rr[c] = PRO == PRO_ADDNORM ? static_cast<const bf16*>(p.R) + arow * p.K : nullptr;
    ro[c] = PRO == PRO_ADDNORM ? static_cast<bf16*>(p.Rout) + arow * p.K : nullptr;
  }

  bf16x8 sa[PF][2], sb[PF][2], sx[PF][2], sg[PF];
  float ss[2] = {0.f, 0.f};

  auto gload = [&](int q, int k0) {
    const int kk = k0 + s_ch * 8;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      sa[q][c] = *reinterpret_cast<const bf16x8*>(xa[c] + kk);
      if constexpr (PRO == PRO_ADDNORM) {
        sx[q][c] = *reinterpret_cast<const bf16x8*>(rr[c] + kk);
      } else if constexpr (PRO == PRO_SILU) {
        sx[q][c] = *reinterpret_cast<const bf16x8*>(xa[c] + p.K + kk);
      }
      sb[q][c] = *reinterpret_cast<const bf16x8*>(wb[c] + kk);
    }
    if constexpr (PRO == PRO_ADDNORM) sg[q] = *reinterpret_cast<const bf16x8*>(LN + kk);
  };
  auto sstore = [&](int q, int buf, int k0) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      bf16x8 av;
      if constexpr (PRO == PRO_PLAIN) {
        av = sa[q][c];
      } else if constexpr (PRO == PRO_ADDNORM) {
        bf16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] = f2bf(bf2f(sa[q][c][j]) + bf2f(sx[q][c][j]));
          const float f = bf2f(s[j]);
          ss[c] += f * f;
          av[j] = f2bf(f * bf2f(sg[q][j]));
        }
        if (tn == 0 && a_ok[c]) *reinterpret_cast<bf16x8*>(ro[c] + k0 + s_ch * 8) = s;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) av[j] = f2bf(silu_bf(bf2f(sa[q][c][j])) * bf2f(sx[q][c][j]));
      }
      lds[buf * 1024 + dswz(s_row[c], s_ch)] = av;
      lds[buf * 1024 + 512 + dswz(s_row[c], s_ch)] = sb[q][c];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma = [&](int buf) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {  // two 32-deep MFMA k-steps per 64-deep tile
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = lds[buf * 1024 + dswz(wm * 32 + i * 16 + fr, ks * 4 + fg)];
        bfr[i] = lds[buf * 1024 + 512 + dswz(wn * 32 + i * 16 + fr, ks * 4 + fg)];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // Epilogue operands are produced by the previous launch: load them now so their latency
  // hides under the K loop instead of adding a dependent round trip at the end.
  float rsc[2][4];        // ss_in row sums of squares of this lane's accumulator rows
  bf16 rold[2][4][2];     // EPI_RESNORM: residual at this lane's outputs
  bf16 lnv[2];            // EPI_RESNORM: next-norm weight at this lane's columns
  // (no per-load "ss_in or 0" select: hipcc would branch around each load and wait on it --
  // without ss_in the loads read valid W bytes and the epilogue ignores them; host-checked)
  const float* ssp = p.ss_in != nullptr ? p.ss_in : static_cast<const float*>(p.W);
  if constexpr (SPL != 1) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + i * 16 + fg * 4 + r;
        const int rowc = row < p.M ? row : 0;
        if constexpr (PRO == PRO_PLAIN) rsc[i][r] = ssp[rowc];
        if constexpr (EPI == EPI_RESNORM) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int col = n0 + wn * 32 + j * 16 + fr;
            rold[i][r][j] = Y[(size_t)rowc * p.ldy + (col < p.N ? col : 0)];
          }
        }
      }
    if constexpr (EPI == EPI_RESNORM) {
      const bf16* lno = static_cast<const bf16*>(p.ln_out);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn * 32 + j * 16 + fr;
        lnv[j] = lno[col < p.N ? col : 0];
      }
    }
  }

  // prologue: PF k-tiles in flight
#pragma unroll
  for (int q = 0; q < PF; ++q) gload(q, kpos(q));
  int t = 0;
  for (; t + PF < nk; t += PF) {  // steady state: consume slot q, refill it PF tiles ahead
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int buf = (t + q) & 1;
      sstore(q, buf, kpos(t + q));
      __syncthreads();
      gload(q, kpos(t + q + PF));
      // pin the refill here: left alone, the scheduler sinks it below the NEXT slot's
      // ds_write (whose vmcnt wait then drains every load: a 1-deep pipeline)
      __builtin_amdgcn_sched_barrier(0);
      mfma(buf);
    }
  }
#pragma unroll
  for (int q = 0; q < PF; ++q) {  // drain: the last PF tiles, no more loads
    const int buf = (t + q) & 1;
    sstore(q, buf, kpos(t + q));
    __syncthreads();
    mfma(buf);
  }

  if constexpr (SPL == 2) {
    // ---- in-launch split-K combine (gdgemm.hip header, SPL 2) ----
    constexpr int NF = 4;  // f32x4 fragments per lane
    const int ntiles = tiles_n * tiles_m;
    constexpr size_t tile_stride = (size_t)NF * 256;
    const size_t zs = (size_t)ntiles * tile_stride;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        p.ws, (short)0, (int)((size_t)S * zs * 16), 0x00020000);
    const size_t mine = ((size_t)kz * ntiles + lt) * tile_stride + tid;  // f32x4 units
#pragma unroll
    for (int f = 0; f < NF; ++f)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[f >> 1][f & 1]), rs,
                                             (int)((mine + (size_t)f * 256) * 16), 0, kDgSc1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
    __syncthreads();
    int* flag = reinterpret_cast<int*>(rowss);  // the plain prologue leaves rowss unused
    if (tid == 0) {
      int* ticket = p.counters + (size_t)lt * kCtrStride;
      const int prev = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == S - 1;
      if (last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (*flag == 0) return;
    // all S slabs (own included), every load issued before any sum; sc1 loads bypass the
    // per-XCD caches a slice on another XCD could not have written through
    const size_t t0 = (size_t)lt * tile_stride + tid;
    f32x4 v[S][NF];
#pragma unroll
    for (int z = 0; z < S; ++z)
#pragma unroll
      for (int f = 0; f < NF; ++f)
        v[z][f] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                       rs, (int)((t0 + (size_t)z * zs + (size_t)f * 256) * 16), 0, kDgSc1));
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      f32x4 s = v[0][f];
#pragma unroll
      for (int z = 1; z < S; ++z) s += v[z][f];
      acc[f >> 1][f & 1] = s;
    }
  }
  if constexpr (PRO == PRO_ADDNORM) {
    // 8 consecutive lanes share a staging row: wave-local butterfly, then one LDS slot/row
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float v = ss[c];
      v += __shfl_xor(v, 1, kWave);
      v += __shfl_xor(v, 2, kWave);
      v += __shfl_xor(v, 4, kWave);
      if ((tid & 7) == 0) {
        rowss[s_row[c]] = v;
        if (SPL == 1 && tn == 0 && a_ok[c])
          p.ws[(size_t)gridDim.y * p.M * p.N + (size_t)kz * p.M + m0 + s_row[c]] = v;
      }
    }
    __syncthreads();
  }
  // epilogue: lane holds rows fg*4 + r, column fr of each 16x16 tile
  const float inv_k = 1.f / (float)p.K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int lrow = wm * 32 + i * 16 + fg * 4 + r;
      const int row = m0 + lrow;
      const bool row_ok = row < p.M;
      if constexpr (SPL == 1) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = n0 + wn * 32 + j * 16 + fr;
          if (row_ok && col < p.N) p.ws[((size_t)kz * p.M + row) * p.N + col] = acc[i][j][r];
        }
        continue;
      }
      float scale = 1.f;
      if constexpr (PRO == PRO_ADDNORM) scale = rsqrtf(rowss[lrow] * inv_k + p.eps);
      if constexpr (PRO == PRO_PLAIN)
        if (p.ss_in != nullptr) scale = rsqrtf(rsc[i][r] * inv_k + p.eps);
      if constexpr (EPI == EPI_STORE) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = n0 + wn * 32 + j * 16 + fr;
          if (row_ok && col < p.N) Y[(size_t)row * p.ldy + col] = f2bf(acc[i][j][r] * scale);
        }
      } else if constexpr (EPI == EPI_RESNORM) {
        bf16* Ao = static_cast<bf16*>(p.Aout);
        float q2 = 0.f;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = n0 + wn * 32 + j * 16 + fr;
          if (row_ok && col < p.N) {
            const bf16 s = f2bf(bf2f(f2bf(acc[i][j][r] * scale)) + bf2f(rold[i][r][j]));
            Y[(size_t)row * p.ldy + col] = s;
            const float f = bf2f(s);
            Ao[(size_t)row * p.N + col] = f2bf(f * bf2f(lnv[j]));
            q2 += f * f;
          }
        }
        // the 16 lanes of this row (same fg) hold its 16 columns of each sub-tile
        q2 += __shfl_xor(q2, 1, kWave);
        q2 += __shfl_xor(q2, 2, kWave);
        q2 += __shfl_xor(q2, 4, kWave);
        q2 += __shfl_xor(q2, 8, kWave);
        if (fr == 0 && row_ok) atomicAdd(p.ss_out + row, q2);
      } else {  // EPI_SILU: j = 0 gate, j = 1 up of feature (n0 + wn*32)/2 + fr
        const int vc = n0 + wn * 32 + fr;
        if (row_ok && vc + 16 < p.N) {
          const float g = bf2f(f2bf(acc[i][0][r] * scale));
          const float u = bf2f(f2bf(acc[i][1][r] * scale));
          Y[(size_t)row * p.ldy + ((n0 + wn * 32) >> 1) + fr] = f2bf(silu_bf(g) * u);
        }
      }
    }
}

// Sum the S fp32 partial slabs [S, M, N] -> bf16, then the same epilogue as the main kernel.
// SCALE: 0 none, 1 ADDNORM (slabs followed by [S, M] partial sums of squares), 2 ss_in[m].
// EPI_RESNORM needs N % 256 == 0 so one wave's 256 consecutive elements share a row.
// S is a template parameter so the S slab loads of an element issue back to back: with a
// runtime trip count hipcc waited on each load before the next (S dependent L2/HBM round
// trips, ~4.5 us at S = 4 in profiles/r1_qwen3_bench_v6_kernel_stats.md).
// IDX: 32-bit element indexing whenever M*N fits (decode sizes always do) -- the 64-bit
// division per element otherwise costs more than the slab reads
template <int SCALE, int EPI, int S, typename IDX = int>
__global__ __launch_bounds__(256) void dgemm_reduce_kernel(DGemmArgs p) {
  const int M = p.M, N = p.N;
  const IDX total = (IDX)M * N / 4;
  const float* ws = p.ws;
  const float* ssw = ws + (size_t)S * M * N;
  bf16* Y = static_cast<bf16*>(p.Y);
  for (IDX i = (IDX)blockIdx.x * 256 + threadIdx.x; i < total; i += (IDX)gridDim.x * 256) {
    const IDX e = i * 4;
    f32x4 part[S];
#pragma unroll
    for (int z = 0; z < S; ++z) part[z] = *reinterpret_cast<const f32x4*>(ws + (size_t)z * M * N + e);
    const int row = (int)(e / N), col = (int)(e - (IDX)row * N);
    float scale = 1.f;
    if constexpr (SCALE == 1) {
      float q[S];
#pragma unroll
      for (int z = 0; z < S; ++z) q[z] = ssw[(size_t)z * M + row];
      float qs = 0.f;
#pragma unroll
      for (int z = 0; z < S; ++z) qs += q[z];
      scale = rsqrtf(qs / (float)p.K + p.eps);
    } else if constexpr (SCALE == 2) {
      scale = rsqrtf(p.ss_in[row] / (float)p.K + p.eps);
    }
    f32x4 s = part[0];
#pragma unroll
    for (int z = 1; z < S; ++z) s += part[z];
    bf16x4* yp = reinterpret_cast<bf16x4*>(Y + (size_t)row * p.ldy + col);
    if constexpr (EPI == EPI_STORE) {
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2bf(s[j] * scale);
      *yp = o;
    } else {  // EPI_RESNORM
      const bf16x4 old = *yp;
      const bf16x4 g = *reinterpret_cast<const bf16x4*>(static_cast<const bf16*>(p.ln_out) + col);
      bf16x4 o, a;
      float q2 = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = f2bf(bf2f(f2bf(s[j] * scale)) + bf2f(old[j]));
        const float f = bf2f(o[j]);
        a[j] = f2bf(f * bf2f(g[j]));
        q2 += f * f;
      }
      *yp = o;
      *reinterpret_cast<bf16x4*>(static_cast<bf16*>(p.Aout) + (size_t)row * N + col) = a;
      q2 = wave_sum(q2);
      if ((threadIdx.x & 63) == 0) atomicAdd(p.ss_out + row, q2);
    }
  }
}

bool dgemm_supported(int M, int N, int K, int splitk, int pf) {
  if (M <= 0 || N <= 0 || K <= 0 || !dgemm_splitk_ok(splitk) || N % 4) return false;
  if (pf != 1 && pf != 2 && pf != 4 && pf != 8) return false;
  if (K % splitk) return false;
  const int kps = K / splitk;
  return kps % (DBK * pf) == 0;
}

bool dgemm_epi_supported(int N, int epi, int splitk) {
  if (epi == EPI_SILU) return splitk == 1 && N % 32 == 0;
  if (epi == EPI_RESNORM) return splitk == 1 || N % 256 == 0;
  return true;
}

template <int PRO, int EPI, int SPL, int S = 1>
static void dgemm_pf(const DGemmArgs& p, dim3 grid, int pf, hipStream_t st) {
  switch (pf) {
    case 8:  // deepest ring: plain operand only (the prologue forms would exceed 256 VGPRs)
      if constexpr (PRO == PRO_PLAIN) dgemm_kernel<PRO, EPI, 8, SPL, S><<<grid, 256, 0, st>>>(p);
      else dgemm_kernel<PRO, EPI, 4, SPL, S><<<grid, 256, 0, st>>>(p);
      break;
    case 4: dgemm_kernel<PRO, EPI, 4, SPL, S><<<grid, 256, 0, st>>>(p); break;
    case 2: dgemm_kernel<PRO, EPI, 2, SPL, S><<<grid, 256, 0, st>>>(p); break;
    default: dgemm_kernel<PRO, EPI, 1, SPL, S><<<grid, 256, 0, st>>>(p); break;
  }
}

template <int SPL, int S = 1>
static void dgemm_main(const DGemmArgs& p, dim3 grid, int pro, int epi, int pf, hipStream_t st) {
  if constexpr (SPL == 2) {  // in-launch combine: plain prologue, every epilogue
    if (epi == EPI_RESNORM) dgemm_pf<PRO_PLAIN, EPI_RESNORM, 2, S>(p, grid, pf, st);
    else if (epi == EPI_SILU) dgemm_pf<PRO_PLAIN, EPI_SILU, 2, S>(p, grid, pf, st);
    else dgemm_pf<PRO_PLAIN, EPI_STORE, 2, S>(p, grid, pf, st);
  } else if (pro == PRO_ADDNORM) {
    dgemm_pf<PRO_ADDNORM, EPI_STORE, SPL>(p, grid, pf, st);
  } else if (pro == PRO_SILU) {
    dgemm_pf<PRO_SILU, EPI_STORE, SPL>(p, grid, pf, st);
  } else if (epi == EPI_RESNORM) {
    dgemm_pf<PRO_PLAIN, EPI_RESNORM, SPL>(p, grid, pf, st);
  } else if (epi == EPI_SILU) {
    if constexpr (SPL == 0) dgemm_pf<PRO_PLAIN, EPI_SILU, 0>(p, grid, pf, st);
  } else {
    dgemm_pf<PRO_PLAIN, EPI_STORE, SPL>(p, grid, pf, st);
  }
}

// Row-parallel RESNORM reduce for decode shapes (N = NI x 1024, M <= 1024): one workgroup per
// output row, every slab / residual / norm-weight load of the row issued before any store, the
// row's sum of squares reduced in LDS and added with ONE atomic per row (the element-parallel
// form issues N/256 same-address atomics per row and waits on its loads element by element:
// 11-14 us for Llama-3-8B's O / down at M = 256, profiles/r3_llama8b_kernel_stats_v2.md).
template <int SCALE, int S, int NI>
__global__ __launch_bounds__(256) void dgemm_reduce_resnorm_row_kernel(DGemmArgs p) {
  __shared__ float scratch[16];
  const int M = p.M, N = p.N, row = blockIdx.x;
  const float* ws = p.ws;
  bf16* Y = static_cast<bf16*>(p.Y);
  const bf16* lno = static_cast<const bf16*>(p.ln_out);
  float scale = 1.f;
  if constexpr (SCALE == 2) scale = rsqrtf(p.ss_in[row] / (float)p.K + p.eps);
  f32x4 acc[NI];
  bf16x4 old[NI], g[NI];
#pragma unroll
  for (int k = 0; k < NI; ++k) {
    const int c = k * 1024 + threadIdx.x * 4;
    const size_t e = (size_t)row * N + c;
    f32x4 part[S];
#pragma unroll
    for (int z = 0; z < S; ++z) part[z] = *reinterpret_cast<const f32x4*>(ws + (size_t)z * M * N + e);
    old[k] = *reinterpret_cast<const bf16x4*>(Y + (size_t)row * p.ldy + c);
    g[k] = *reinterpret_cast<const bf16x4*>(lno + c);
    acc[k] = part[0];
#pragma unroll
    for (int z = 1; z < S; ++z) acc[k] += part[z];
  }
  float q2 = 0.f;
  bf16* Ao = static_cast<bf16*>(p.Aout);
#pragma unroll
  for (int k = 0; k < NI; ++k) {
    const int c = k * 1024 + threadIdx.x * 4;
    bf16x4 o, a;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = f2bf(bf2f(f2bf(acc[k][j] * scale)) + bf2f(old[k][j]));
      const float f = bf2f(o[j]);
      a[j] = f2bf(f * bf2f(g[k][j]));
      q2 += f * f;
    }
    *reinterpret_cast<bf16x4*>(Y + (size_t)row * p.ldy + c) = o;
    *reinterpret_cast<bf16x4*>(Ao + (size_t)row * N + c) = a;
  }
  q2 = block_sum(q2, scratch);
  if (threadIdx.x == 0) atomicAdd(p.ss_out + row, q2);
}

template <int SCALE, int S>
static bool reduce_row_ni(const DGemmArgs& p, hipStream_t st) {
  switch (p.N / 1024) {
    case 1: dgemm_reduce_resnorm_row_kernel<SCALE, S, 1><<<p.M, 256, 0, st>>>(p); return true;
    case 2: dgemm_reduce_resnorm_row_kernel<SCALE, S, 2><<<p.M, 256, 0, st>>>(p); return true;
    case 4: dgemm_reduce_resnorm_row_kernel<SCALE, S, 4><<<p.M, 256, 0, st>>>(p); return true;
    case 8: dgemm_reduce_resnorm_row_kernel<SCALE, S, 8><<<p.M, 256, 0, st>>>(p); return true;
    default: return false;
  }
}

template <int SCALE>
static bool reduce_row(const DGemmArgs& p, int splitk, hipStream_t st) {
  if (p.N % 1024 || p.M > 1024) return false;
  switch (splitk) {
    case 2: return reduce_row_ni<SCALE, 2>(p, st);
    case 4: return reduce_row_ni<SCALE, 4>(p, st);
    case 8: return p.N <= 4096 && reduce_row_ni<SCALE, 8>(p, st);  // keep the slab registers < 256
    default: return false;
  }
}

template <int SCALE, int EPI, typename IDX>
static void reduce_s_idx(const DGemmArgs& p, int splitk, int blocks, hipStream_t st) {
  switch (splitk) {
    case 2: dgemm_reduce_kernel<SCALE, EPI, 2, IDX><<<blocks, 256, 0, st>>>(p); break;
    case 4: dgemm_reduce_kernel<SCALE, EPI, 4, IDX><<<blocks, 256, 0, st>>>(p); break;
    case 8: dgemm_reduce_kernel<SCALE, EPI, 8, IDX><<<blocks, 256, 0, st>>>(p); break;
    default: dgemm_reduce_kernel<SCALE, EPI, 16, IDX><<<blocks, 256, 0, st>>>(p); break;
  }
}

template <int SCALE, int EPI>
static void reduce_s(const DGemmArgs& p, int splitk, int blocks, hipStream_t st) {
  if ((long)p.M * p.N + 4L * blocks * 256 < (1L << 31))
    reduce_s_idx<SCALE, EPI, int>(p, splitk, blocks, st);
  else
    reduce_s_idx<SCALE, EPI, long>(p, splitk, blocks, st);
}

bool dgemm_splitk_ok(int splitk) {
  return splitk == 1 || splitk == 2 || splitk == 4 || splitk == 8 || splitk == 16;
}

void launch_dgemm_reduce(const DGemmArgs& p, int pro, int splitk, hipStream_t st) {
  long blocks = ((long)p.M * p.N / 4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  const int b = (int)blocks;
  const int scale = pro == PRO_ADDNORM ? 1 : (pro == PRO_PLAIN && p.ss_in ? 2 : 0);
  if (p.epi == EPI_RESNORM) {
    if (scale == 2) {
      if (!reduce_row<2>(p, splitk, st)) reduce_s<2, EPI_RESNORM>(p, splitk, b, st);
    } else {
      if (!reduce_row<0>(p, splitk, st)) reduce_s<0, EPI_RESNORM>(p, splitk, b, st);
    }
  } else if (scale == 1) {
    reduce_s<1, EPI_STORE>(p, splitk, b, st);
  } else if (scale == 2) {
    reduce_s<2, EPI_STORE>(p, splitk, b, st);
  } else {
    reduce_s<0, EPI_STORE>(p, splitk, b, st);
  }
}

void launch_dgemm(const DGemmArgs& a, int pro, int splitk, int pf, hipStream_t st) {
  if (a.M == 0 || a.N == 0) return;
  DGemmArgs p = a;
  p.kps = a.K / splitk;
  if (pro != PRO_PLAIN) p.epi = EPI_STORE;  // prologue forms have the plain store epilogue
  if (pro == PRO_PLAIN && p.bn > 0) {        // LDS-DMA (global_load_lds) ring variant
    launch_gdgemm(p, splitk, st);
    return;
  }
  const int tiles = ((a.M + DBM - 1) / DBM) * ((a.N + DBN - 1) / DBN);
  dim3 grid(tiles, splitk);
  if (splitk > 1 && p.counters != nullptr && pro == PRO_PLAIN &&
      (splitk == 2 || splitk == 4 || splitk == 8)) {  // in-launch combine
    if (splitk == 2) dgemm_main<2, 2>(p, grid, pro, p.epi, pf, st);
    else if (splitk == 4) dgemm_main<2, 4>(p, grid, pro, p.epi, pf, st);
    else dgemm_main<2, 8>(p, grid, pro, p.epi, pf, st);
  } else if (splitk > 1) {
    dgemm_main<1>(p, grid, pro, p.epi, pf, st);
    launch_dgemm_reduce(p, pro, splitk, st);
  } else {
    dgemm_main<0>(p, grid, pro, p.epi, pf, st);
  }
}

}  // namespace akap
