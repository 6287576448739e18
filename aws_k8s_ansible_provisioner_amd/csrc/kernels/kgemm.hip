// Narrow-output decode GEMM with the K split INSIDE the workgroup, for gfx950:
//   Y[M,N] = X[M,K] . W[N,K]^T   (N = d_model: the O and down projections, N = 1,024 for
//   Qwen3-0.6B) with dgemm.hip's epilogues (plain store / residual + next-norm), optional
//   ss_in row scale.
//
// Why: at M = 256, N = 1,024 a 64 x 64 output tiling has only 64 tiles, so the decode GEMMs
// split K over 4 workgroups to fill the chip and pay for it with fp32 partial slabs and a
// separate reduce launch (dgemm_reduce_kernel: ~4.9 us per call + a ~1.5 us kernel boundary,
// profiles/r2_pmc_decode.md) -- ~10.6 us for a projection whose weights stream in ~1 us.
// Here a workgroup owns a small BM x 32 output tile (BM = 16 | 32: 256 workgroups at M = 256,
// N = 1,024) and its 4 waves take interleaved 64-deep slices of every 256-deep K stage; the
// four partial tiles are summed through LDS at the end, so there are no global partials and
// no second launch.
//
// Staging: one K stage = (BM + 32) rows x 256 k of bf16 (24 / 32 KB) by global_load_lds
// (LDS-DMA, 16 B per lane, lane-linear destination) into an NS = 4 slot ring -> three stages
// in flight; counted `s_waitcnt vmcnt` + raw s_barrier per stage.  LDS row = 32 chunks of 16 B
// (512 B: every row starts on the same bank); the low four chunk bits are XORed with row & 15
// (on the DMA source address and on the fragment reads -- cdna_hip_programming.md rule 21), so
// the 16 lanes of each ds_read_b128 lane group (rows 0-3, 12-15 at chunk c, rows 4-11 at c+1)
// land on 16 distinct 16-B bank positions: conflict-free (XOR with row & 7 measured 48 %
// bank-conflict cycles, profiles/r2_pmc_decode_v2.md).
#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int KBN = 32;    // output columns per workgroup
constexpr int KST = 256;   // K per stage (4 waves x 64)

__device__ __forceinline__ int kswz(int row, int chunk) { return row * 32 + (chunk ^ (row & 15)); }

__device__ __forceinline__ void kglds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0,
                                   0);
}
__device__ __forceinline__ void kglds16_nt(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0,
                                   2);
}

template <int N_>
__device__ __forceinline__ void kwait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

// KNS = 4 ring slots: 3 stages (96 KB) in flight (a 5-slot ring lost 0.5 % end to end and was
// removed, profiles/r3_gemm_m256_deep.log)
template <int BM, int EPI, int KNS>
__global__ __launch_bounds__(256, 1) void kgemm_kernel(DGemmArgs p) {
  constexpr int ROWS = BM + KBN;            // staged rows per stage (X rows, then W rows)
  constexpr int SU = ROWS * 32;             // 16-B units per slot
  constexpr int G = ROWS * 32 / 64 / 4;     // DMA instructions per wave per stage
  constexpr int MI = BM / 16;               // 16-row MFMA tiles
  constexpr int LDS_UNITS = KNS * SU;
  static_assert(4 * BM * KBN * 4 <= LDS_UNITS * 16, "combine buffer fits in the ring");
  __shared__ bf16x8 lds[LDS_UNITS];

  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = p.N / KBN;
  const int lt = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = lt / tiles_m, tm = lt % tiles_m;  // a column tile's row tiles share an XCD
  const int m0 = tm * BM, n0 = tn * KBN;
  const int nst = p.K / KST;
  const int st0 = gemm_stagger0(p.stag, tm, tn, nst);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const bf16* X = static_cast<const bf16*>(p.X);
  const bf16* Wt = static_cast<const bf16*>(p.W);
  bf16* Y = static_cast<bf16*>(p.Y);

  // DMA instruction j (= w * G + i) fills slot units [64 j, 64 j + 64): rows 2j, 2j+1
  const bf16* src[G];
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const int u = (w * G + i) * 64 + lane;
    const int row = u >> 5;
    const int lchunk = (u & 31) ^ (row & 15);
    const bf16* base;
    if (row < BM) {
      const int m = m0 + row;
      base = X + (size_t)(m < p.M ? m : 0) * p.ldx;
    } else {
      base = Wt + (size_t)(n0 + row - BM) * p.ldw;
    }
    src[i] = base + lchunk * 8;
  }
  auto issue = [&](int st) {
    bf16x8* slot = lds + (st % KNS) * SU;
    int ks = st + st0;
    if (ks >= nst) ks -= nst;
    const int k0 = ks * KST;
#pragma unroll
    for (int i = 0; i < G; ++i) {
      // instruction (w, i) stages rows 2 (w G + i) and + 1: X rows below BM, weight rows above
      // (wave-uniform), the weights non-temporal only when asked for (p.ntw == 1)
      if (p.ntw == 1 && (w * G + i) * 2 >= BM) kglds16_nt(src[i] + k0, slot + (w * G + i) * 64);
      else kglds16(src[i] + k0, slot + (w * G + i) * 64);
    }
  };

  // epilogue operands of the previous launch, loaded under the K loop
  const int er = tid >> 3;          // combine / epilogue: row er (of 32), cols 4 * (tid & 7)
  const int ec = (tid & 7) * 4;
  const int erow = m0 + er;
  const bool e_ok = er < BM && erow < p.M;
  const int erc = e_ok ? erow : 0;
  float rs = 0.f;
  bf16x4 rold = {0, 0, 0, 0}, lnv = {0, 0, 0, 0};
  if (p.ss_in != nullptr) rs = p.ss_in[erc];
  if constexpr (EPI == EPI_RESNORM) {
    rold = *reinterpret_cast<const bf16x4*>(Y + (size_t)erc * p.ldy + n0 + ec);
    lnv = *reinterpret_cast<const bf16x4*>(static_cast<const bf16*>(p.ln_out) + n0 + ec);
  }

  f32x4 acc[MI][2];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < KNS - 1; ++s)
    if (s < nst) issue(s);
  for (int t = 0; t < nst; ++t) {
    if (t + KNS - 2 < nst) kwait_vm<G * (KNS - 2)>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage t landed for every wave; slot t-1 is free
    if (t + KNS - 1 < nst) issue(t + KNS - 1);
    const bf16x8* slot = lds + (t % KNS) * SU;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = w * 8 + ks * 4 + fg;  // this wave's 64-k slice of the stage
      bf16x8 af[MI], bfr[2];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = slot[kswz(i * 16 + fr, ch)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = slot[kswz(BM + j * 16 + fr, ch)];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  // ---- sum the 4 waves' partial tiles through LDS: part[w][row][32] fp32 ----
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // ring no longer read
  float* part = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        part[(w * BM + i * 16 + fg * 4 + r) * KBN + j * 16 + fr] = acc[i][j][r];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (er >= BM) return;  // BM = 16: threads of rows 16..31 have no work
  f32x4 v = *reinterpret_cast<const f32x4*>(&part[er * KBN + ec]);
#pragma unroll
  for (int ww = 1; ww < 4; ++ww) v += *reinterpret_cast<const f32x4*>(&part[(ww * BM + er) * KBN + ec]);
  const float scale = p.ss_in != nullptr ? rsqrtf(rs / (float)p.K + p.eps) : 1.f;
  if constexpr (EPI == EPI_STORE) {
    if (!e_ok) return;
    bf16x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = f2bf(v[q] * scale);
    *reinterpret_cast<bf16x4*>(Y + (size_t)erow * p.ldy + n0 + ec) = o;
  } else {  // EPI_RESNORM: residual += y; Aout = residual * ln_out; ss_out += row sum of squares
    bf16x4 o, a;
    float q2 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      o[q] = f2bf(bf2f(f2bf(v[q] * scale)) + bf2f(rold[q]));
      const float f = bf2f(o[q]);
      a[q] = f2bf(f * bf2f(lnv[q]));
      q2 += f * f;
    }
    // the 8 threads of a row are consecutive lanes
    q2 += __shfl_xor(q2, 1, 8);
    q2 += __shfl_xor(q2, 2, 8);
    q2 += __shfl_xor(q2, 4, 8);
    if (!e_ok) return;
    *reinterpret_cast<bf16x4*>(Y + (size_t)erow * p.ldy + n0 + ec) = o;
    *reinterpret_cast<bf16x4*>(static_cast<bf16*>(p.Aout) + (size_t)erow * p.N + n0 + ec) = a;
    if ((tid & 7) == 0) atomicAdd(p.ss_out + erow, q2);
  }
}

bool kgemm_supported(int M, int N, int K, int bm) {
  return M > 0 && (bm == 16 || bm == 32) && N % KBN == 0 && K >= KST && K % KST == 0;
}

void launch_kgemm(const DGemmArgs& p, int bm, hipStream_t st) {
  if (p.M == 0) return;
  constexpr int KNS = 4;
  const int grid = ((p.M + bm - 1) / bm) * (p.N / KBN);
  if (bm == 16) {
    if (p.epi == EPI_RESNORM) kgemm_kernel<16, EPI_RESNORM, KNS><<<grid, 256, 0, st>>>(p);
    else kgemm_kernel<16, EPI_STORE, KNS><<<grid, 256, 0, st>>>(p);
  } else {
    if (p.epi == EPI_RESNORM) kgemm_kernel<32, EPI_RESNORM, KNS><<<grid, 256, 0, st>>>(p);
    else kgemm_kernel<32, EPI_STORE, KNS><<<grid, 256, 0, st>>>(p);
  }
}

}  // namespace akap
