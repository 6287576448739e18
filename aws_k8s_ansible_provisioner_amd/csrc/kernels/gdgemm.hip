// Decode GEMM with LDS-DMA operand staging for gfx950:  Y[M,N] = X[M,K] . W[N,K]^T
// (plain prologue + the dgemm.hip epilogues: store / residual+next-norm / SwiGLU, optional
// ss_in row scale, split-K partials reduced by dgemm.hip's reduce pass).
//
// Why: at decode sizes these GEMMs are bound by how many bytes per second each CU can pull
// through its vector-load path; register staging (dgemm.hip) tops out at ~30-36 GB/s per CU,
// while global_load_lds writes LDS directly (no VGPR round trip, no ds_write pass) and a CU
// can take in far more (MI355X_MICROARCH.md price table rows ldsdma-fill / ring-gemm).
//
// Structure: 64 x BN output tile (BN 64 | 128), 4 waves as 2 (M) x 2 (N), BK = 64.  An LDS
// ring of NS k-step slots [A 64 rows | W BN rows] x 128 B; NS-1 k-steps of global_load_lds
// in flight.  Per k-step: counted `s_waitcnt vmcnt` for this step's DMAs, raw s_barrier (never
// __syncthreads: its fence would drain every DMA in flight), refill the slot consumed one
// step earlier, then ds_read fragments + MFMA.  LDS image: linear DMA destination, XOR swizzle
// applied to the per-lane SOURCE address and to the fragment reads (the same involution,
// cdna_hip_programming.md rule 21).
#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int GBM = 64, GBK = 64;

__device__ __forceinline__ int gswz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0,
                                   0);
}

template <int N_>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N_ >= 63) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

template <int BN, int NS, int EPI, bool SPLIT>
__global__ __launch_bounds__(256, 2) void gdgemm_kernel(DGemmArgs p) {
  constexpr int SU = (GBM + BN) * 8;      // slot size in 16-B units
  constexpr int JN = BN / 32;             // 16-col MFMA tiles per wave (wave tile 32 x BN/2)
  constexpr int GA = 2, GW = BN / 32;     // DMA instructions per wave per k-step (A / W)
  constexpr int G = GA + GW;
  __shared__ bf16x8 lds[NS * SU];

  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles_m = (p.M + GBM - 1) / GBM;
  const int lt = xcd_remap(blockIdx.x, tiles_n * tiles_m);
  const int tn = lt / tiles_m, tm = lt % tiles_m;
  const int m0 = tm * GBM, n0 = tn * BN;
  const int kz = blockIdx.y;
  const int kbeg = kz * p.kps;
  const int nk = p.kps / GBK;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const bf16* X = static_cast<const bf16*>(p.X);
  const bf16* W = static_cast<const bf16*>(p.W);
  bf16* Y = static_cast<bf16*>(p.Y);

  // per-lane DMA sources: instruction covers 8 rows x 128 B; lane -> row L/8, LDS chunk L%8
  // holding logical chunk (L%8) ^ (L/8)  (row & 7 == L/8 since every instruction starts on a
  // multiple of 8 rows)
  const int lr = lane >> 3, lc = (lane & 7) ^ (lane >> 3);
  const bf16* asrc[GA];
  const bf16* wsrc[GW];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int row = m0 + (w * GA + i) * 8 + lr;
    asrc[i] = X + (size_t)(row < p.M ? row : 0) * p.ldx + lc * 8;
  }
#pragma unroll
  for (int i = 0; i < GW; ++i) {
    const int v = n0 + (w * GW + i) * 8 + lr;
    int wrow = v < p.N ? v : 0;
    if constexpr (EPI == EPI_SILU)
      wrow = v < p.N ? ((v >> 4) & 1) * (p.N >> 1) + (v >> 5) * 16 + (v & 15) : 0;
    wsrc[i] = W + (size_t)wrow * p.ldw + lc * 8;
  }
  auto issue = [&](int step) {  // DMA k-step `step` into its ring slot
    bf16x8* slot = lds + (step % NS) * SU;
    const int k0 = kbeg + step * GBK;
#pragma unroll
    for (int i = 0; i < GA; ++i) glds16(asrc[i] + k0, slot + (w * GA + i) * 64);
#pragma unroll
    for (int i = 0; i < GW; ++i) glds16(wsrc[i] + k0, slot + GBM * 8 + (w * GW + i) * 64);
  };

  // epilogue operands from the previous launch: load before the loop (hidden under it)
  float rsc[2][4];
  bf16 rold[2][4][JN];
  bf16 lnv[JN];
  const float* ssp = p.ss_in != nullptr ? p.ss_in : static_cast<const float*>(p.W);
  if constexpr (!SPLIT) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + i * 16 + fg * 4 + r;
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

  f32x4 acc[2][JN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: NS-1 k-steps in flight (host: nk >= NS - 1)
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) issue(s);
  for (int t = 0; t < nk; ++t) {
    // retire this thread's DMAs of step t: the later steps issued so far stay in flight
    if (t + NS - 2 < nk) wait_vm<G * (NS - 2)>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMAs of step t landed; slot t-1 is free
    if (t + NS - 1 < nk) issue(t + NS - 1);
    const bf16x8* slot = lds + (t % NS) * SU;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[2], bfr[JN];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = slot[gswz(wm * 32 + i * 16 + fr, ks * 4 + fg)];
#pragma unroll
      for (int j = 0; j < JN; ++j)
        bfr[j] = slot[GBM * 8 + gswz(wn * (BN / 2) + j * 16 + fr, ks * 4 + fg)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  // epilogue: lane holds rows wm*32 + i*16 + fg*4 + r, column fr of each 16-col sub-tile
  const float inv_k = 1.f / (float)p.K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm * 32 + i * 16 + fg * 4 + r;
      const bool row_ok = row < p.M;
      if constexpr (SPLIT) {
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

bool gdgemm_supported(int M, int N, int K, int splitk, int bn) {
  if (bn != 64 && bn != 128) return false;
  if (M <= 0 || N <= 0 || K <= 0 || splitk < 1 || N % 4 || K % splitk) return false;
  const int kps = K / splitk;
  return kps % GBK == 0 && kps / GBK >= 3;  // ring prologue keeps up to 3 k-steps in flight
}

template <int BN, int NS, bool SPL>
static void gdgemm_epi(const DGemmArgs& p, dim3 grid, hipStream_t st) {
  if (p.epi == EPI_RESNORM) gdgemm_kernel<BN, NS, EPI_RESNORM, SPL><<<grid, 256, 0, st>>>(p);
  else if (p.epi == EPI_SILU) {
    if constexpr (!SPL) gdgemm_kernel<BN, NS, EPI_SILU, false><<<grid, 256, 0, st>>>(p);
  } else gdgemm_kernel<BN, NS, EPI_STORE, SPL><<<grid, 256, 0, st>>>(p);
}

void launch_gdgemm(const DGemmArgs& p, int splitk, hipStream_t st) {
  const int tiles = ((p.M + GBM - 1) / GBM) * ((p.N + p.bn - 1) / p.bn);
  dim3 grid(tiles, splitk);
  // NS = 4 (64-col: 4 x 16 KB) / 3 (128-col: 3 x 24 KB): two blocks fit a CU's 160 KB LDS
  if (splitk > 1) {
    if (p.bn == 128) gdgemm_epi<128, 3, true>(p, grid, st);
    else gdgemm_epi<64, 4, true>(p, grid, st);
    launch_dgemm_reduce(p, PRO_PLAIN, splitk, st);
  } else {
    if (p.bn == 128) gdgemm_epi<128, 3, false>(p, grid, st);
    else gdgemm_epi<64, 4, false>(p, grid, st);
  }
}

}  // namespace akap
