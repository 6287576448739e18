// Wide-row decode GEMM for gfx950:  Y[M,N] = X[M,K] . W[N,K]^T  for M <= 256 and large N --
// the LM head (N = vocab slice: 151,936 x 1,024 = 311 MB for Qwen3-0.6B, 128,256 x 4,096 =
// 1.05 GB for Llama-3-8B) and other weight-streaming projections.
//
// Why a separate kernel: with the decode GEMMs' 64-row tiles (dgemm.hip / gdgemm.hip) a
// 256-row batch splits into 4 row tiles, so every weight byte crosses L2 -> CU four times
// and the launch is L2-bandwidth bound (hipBLASLt's 160x256 macro-tile: 136 us for the
// Qwen3 LM head at M = 256 = 2.3 TB/s of weights, profiles/r1_qwen3_bench_v6_kernel_stats.md).
// Here ONE workgroup owns all (up to 256) rows of its column tile, so the weights stream
// from HBM exactly once and only the small, L2-resident activation block is re-read.
//
// Geometry (512 threads, 8 waves, one workgroup per CU, BK = 64):
//   WM = 4: 256 x 128 tile, waves 4 (M) x 2 (N), wave tile 64 x 64
//   WM = 2: 128 x 256 tile, waves 2 (M) x 4 (N), wave tile 64 x 64
//   WM = 1:  64 x 256 tile, waves 1 (M) x 8 (N), wave tile 64 x 32
// Operands are staged by global_load_lds (LDS-DMA) into an NS = 3 slot ring (two k-steps
// in flight, <= 144 KB), XOR-swizzled on the per-lane SOURCE address and on the fragment
// reads (cdna_hip_programming.md rule 21); counted `s_waitcnt vmcnt` + raw s_barrier per
// k-step (a __syncthreads would drain every DMA in flight); v_mfma_f32_16x16x32_bf16.
// Epilogue: the wave tile goes through LDS (the ring is free by then) so the bf16 output is
// written as whole 16-byte row segments instead of 2-byte fragment scatters -- at M = 256
// the LM head writes 78 MB of logits.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int WBK = 64;
constexpr int WNS = 3;

template <int WM>
struct WCfg {
  static constexpr int BM = 64 * WM;
  static constexpr int WN = 8 / WM;            // waves along N
  static constexpr int BN = WM == 4 ? 128 : 256;
  static constexpr int WC = BN / WN;           // columns per wave: 64 | 64 | 32
  static constexpr int JN = WC / 16;           // 16-col MFMA tiles per wave
  static constexpr int GA = WM;                // X DMA instructions per wave per k-step
  static constexpr int GW = BN / 64;           // W DMA instructions per wave per k-step
  static constexpr int G = GA + GW;
  static constexpr int SU = (BM + BN) * 8;     // ring slot in 16-B units
  static constexpr int EP = WC + 8;            // epilogue LDS row pitch (bf16), de-conflicted
};

__device__ __forceinline__ int wswz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }

template <int AUX = 0>
__device__ __forceinline__ void wglds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0,
                                   AUX);
}

template <int N_>
__device__ __forceinline__ void wwait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

// NTW: the weight stream's DMAs carry the non-temporal policy (aux = 2): every weight byte is
// read by exactly one workgroup, once
template <int WM, bool NTW = false>
__global__ __launch_bounds__(512, 2) void wgemm_kernel(WGemmArgs p) {
  using C = WCfg<WM>;
  // ONE __shared__ object (cdna_hip_programming.md "Projection GEMM at M = 256" item 4a)
  __shared__ bf16x8 lds[WNS * C::SU];

  const int tn = blockIdx.x, tm = blockIdx.y;
  const int m0 = tm * C::BM, n0 = tn * C::BN;
  const int nk = p.K / WBK;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / C::WN, wn = w % C::WN;
  const int fr = lane & 15, fg = lane >> 4;
  const bf16* X = static_cast<const bf16*>(p.X);
  const bf16* W = static_cast<const bf16*>(p.W);

  // per-lane DMA sources: one instruction = 8 rows x 128 B; lane -> row L/8, LDS chunk L%8
  // holding logical chunk (L%8) ^ (L/8).  Rows past M / N re-read row 0 (never stored).
  const int lr = lane >> 3, lc = (lane & 7) ^ (lane >> 3);
  const bf16* asrc[C::GA];
  const bf16* wsrc[C::GW];
#pragma unroll
  for (int i = 0; i < C::GA; ++i) {
    const int row = m0 + (w * C::GA + i) * 8 + lr;
    asrc[i] = X + (size_t)(row < p.M ? row : 0) * p.ldx + lc * 8;
  }
#pragma unroll
  for (int i = 0; i < C::GW; ++i) {
    const int v = n0 + (w * C::GW + i) * 8 + lr;
    wsrc[i] = W + (size_t)(v < p.N ? v : 0) * p.ldw + lc * 8;
  }
  auto issue = [&](int step) {
    bf16x8* slot = lds + (step % WNS) * C::SU;
    const int k0 = step * WBK;
#pragma unroll
    for (int i = 0; i < C::GA; ++i) wglds16(asrc[i] + k0, slot + (w * C::GA + i) * 64);
#pragma unroll
    for (int i = 0; i < C::GW; ++i)
      wglds16<NTW ? 2 : 0>(wsrc[i] + k0, slot + C::BM * 8 + (w * C::GW + i) * 64);
  };

  f32x4 acc[4][C::JN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < C::JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < WNS - 1; ++s)
    if (s < nk) issue(s);
  for (int t = 0; t < nk; ++t) {
    // retire this thread's DMAs of step t (step t+1 stays in flight when it exists)
    if (t + 1 < nk) wwait_vm<C::G>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMAs of step t landed; slot t-1 is free
    if (t + WNS - 1 < nk) issue(t + WNS - 1);
    const bf16x8* slot = lds + (t % WNS) * C::SU;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4], bfr[C::JN];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = slot[wswz(wm * 64 + i * 16 + fr, ks * 4 + fg)];
#pragma unroll
      for (int j = 0; j < C::JN; ++j)
        bfr[j] = slot[C::BM * 8 + wswz(wn * C::WC + j * 16 + fr, ks * 4 + fg)];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < C::JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  // ---- epilogue: accumulators -> bf16 wave tile in LDS -> 16-byte row-segment stores ----
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // every wave is done reading the ring
  bf16* et = reinterpret_cast<bf16*>(lds) + (size_t)w * 64 * C::EP;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < C::JN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) et[(i * 16 + fg * 4 + r) * C::EP + j * 16 + fr] = f2bf(acc[i][j][r]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local tile: no barrier needed
  bf16* Y = static_cast<bf16*>(p.Y);
  constexpr int CPR = C::WC / 8;  // 16-byte chunks per wave-tile row
#pragma unroll
  for (int e = lane; e < 64 * CPR; e += 64) {
    const int rr = e / CPR, cc = e % CPR;
    const int row = m0 + wm * 64 + rr;
    const int col = n0 + wn * C::WC + cc * 8;
    if (row >= p.M || col >= p.N) continue;
    const bf16* src = et + rr * C::EP + cc * 8;
    bf16* dst = Y + (size_t)row * p.ldy + col;
    if (col + 8 <= p.N) {
      bf16x8 v;
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = src[q];
      *reinterpret_cast<bf16x8*>(dst) = v;
    } else {
      for (int q = 0; q < p.N - col; ++q) dst[q] = src[q];
    }
  }
}

// ------------------------------------------------------------------------------------------
// Wide form for 129..256 rows: 256 x 256 tiles.  The LM head at M = 256 is bound by the L2 ->
// CU traffic of all workgroups together (~9 TB/s chip-wide for decode-GEMM tile streams,
// profiles/r6_decode_gemm_ingress.md), and with 256 x 128 tiles two thirds of that traffic is
// the 512 KB activation block re-read by every one of the 1,187 column tiles (911 MB per call
// for Qwen3-0.6B = the measured ~101 us).  256-wide tiles halve the re-reads (594 tiles, 594 MB).
// 8 waves as 4 (M) x 2 (N), wave tile 64 x 128 (128 accumulator registers); 32-deep k-steps
// (rows of 64 B, chunk c stored at c ^ g((row >> 2) & 3), g = {0, 2, 3, 1}: conflict-free for
// ds_read_b128 fragment reads, see pgemm.hip pu_swz) through a 4-slot ring of 32 KB, three
// k-steps in flight; one DMA instruction = 16 rows x 64 B.
__device__ __forceinline__ int ww_swz(int row, int c) {
  return row * 4 + (c ^ ((0x1320 >> (4 * ((row >> 2) & 3))) & 3));
}

template <bool NTW>
__global__ __launch_bounds__(512, 1) void wgemm_wide_kernel(WGemmArgs p) {
  constexpr int BM = 256, BN = 256, BK = 32, NS = 4;
  constexpr int SU = (BM + BN) * 4;             // 16-B units per slot (32 KB)
  constexpr int GA = BM / 16 / 8, GW = BN / 16 / 8;  // DMA instructions per wave per k-step
  constexpr int G = GA + GW;
  constexpr int WC = 128, JN = 8, EP = WC + 8;  // wave tile 64 x 128; epilogue row pitch
  constexpr int RING = NS * SU, EPI_UNITS = 8 * 64 * EP / 8;
  __shared__ bf16x8 lds[RING > EPI_UNITS ? RING : EPI_UNITS];

  const int tn = blockIdx.x;
  const int n0 = tn * BN;
  const int nk = p.K / BK;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const bf16* X = static_cast<const bf16*>(p.X);
  const bf16* W = static_cast<const bf16*>(p.W);
  // lane -> row lane / 4 of the instruction's 16, LDS chunk lane % 4 holding logical chunk
  // (lane % 4) ^ g((row >> 2) & 3) (instructions start on multiples of 16 rows)
  const int lr = lane >> 2;
  const int lc = (lane & 3) ^ ((0x1320 >> (4 * ((lr >> 2) & 3))) & 3);
  const bf16* asrc[GA];
  const bf16* wsrc[GW];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int row = (w * GA + i) * 16 + lr;
    asrc[i] = X + (size_t)(row < p.M ? row : 0) * p.ldx + lc * 8;
  }
#pragma unroll
  for (int i = 0; i < GW; ++i) {
    const int v = n0 + (w * GW + i) * 16 + lr;
    wsrc[i] = W + (size_t)(v < p.N ? v : 0) * p.ldw + lc * 8;
  }
  auto issue = [&](int step) {
    bf16x8* slot = lds + (step % NS) * SU;
    const int k0 = step * BK;
#pragma unroll
    for (int i = 0; i < GA; ++i) wglds16(asrc[i] + k0, slot + (w * GA + i) * 64);
#pragma unroll
    for (int i = 0; i < GW; ++i)
      wglds16<NTW ? 2 : 0>(wsrc[i] + k0, slot + BM * 4 + (w * GW + i) * 64);
  };

  f32x4 acc[4][JN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s);
  for (int t = 0; t < nk; ++t) {
    // retire step t (steps t+1, t+2 stay in flight when they exist)
    if (t + 2 < nk) wwait_vm<2 * G>();
    else if (t + 1 < nk) wwait_vm<G>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMAs of step t landed; slot t-1 is free
    if (t + NS - 1 < nk) issue(t + NS - 1);
    const bf16x8* slot = lds + (t % NS) * SU;
    bf16x8 af[4], bfr[JN];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = slot[ww_swz(wm * 64 + i * 16 + fr, fg)];
#pragma unroll
    for (int j = 0; j < JN; ++j) bfr[j] = slot[BM * 4 + ww_swz(wn * WC + j * 16 + fr, fg)];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  }

  // ---- epilogue: as wgemm_kernel (wave tile through LDS, 16-byte row-segment stores) ----
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  bf16* et = reinterpret_cast<bf16*>(lds) + (size_t)w * 64 * EP;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) et[(i * 16 + fg * 4 + r) * EP + j * 16 + fr] = f2bf(acc[i][j][r]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bf16* Y = static_cast<bf16*>(p.Y);
  constexpr int CPR = WC / 8;
  for (int e = lane; e < 64 * CPR; e += 64) {
    const int rr = e / CPR, cc = e % CPR;
    const int row = wm * 64 + rr;
    const int col = n0 + wn * WC + cc * 8;
    if (row >= p.M || col >= p.N) continue;
    const bf16* src = et + rr * EP + cc * 8;
    bf16* dst = Y + (size_t)row * p.ldy + col;
    if (col + 8 <= p.N) {
      bf16x8 v;
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = src[q];
      *reinterpret_cast<bf16x8*>(dst) = v;
    } else {
      for (int q = 0; q < p.N - col; ++q) dst[q] = src[q];
    }
  }
}

// AKAP_WGEMM_WIDE: 1 -> the 256 x 256 form for 129..256 rows (K % 32 == 0), 0 -> 256 x 128
static int wgemm_wide() {
  static const int v = [] {
    const char* e = std::getenv("AKAP_WGEMM_WIDE");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

int wgemm_rows(int M) { return M <= 64 ? 1 : (M <= 128 ? 2 : 4); }

bool wgemm_supported(int M, int N, int K, int ldx, int ldw, int ldy) {
  return M > 0 && N > 0 && K >= WBK && K % WBK == 0 && ldx % 8 == 0 && ldw % 8 == 0 &&
         ldy % 8 == 0;
}

void launch_wgemm(const WGemmArgs& p, hipStream_t st) {
  if (p.M == 0 || p.N == 0) return;
  const int wmr = wgemm_rows(p.M);
  const int bm = 64 * wmr, bn = wmr == 4 ? 128 : 256;
  dim3 grid((p.N + bn - 1) / bn, (p.M + bm - 1) / bm);
  // non-temporal weight DMAs by default (AKAP_WGEMM_NT=0 disables): measured on MI355X,
  // Qwen3 LM head M=256 111.5 -> 108.2 us, Llama-3-8B LM head M=16/128 232/257 -> 205/226 us
  // (profiles/r2_wgemm_nt.log)
  static const bool nt = [] {
    const char* e = std::getenv("AKAP_WGEMM_NT");
    return e == nullptr || std::atoi(e) != 0;
  }();
  if (wmr == 4 && p.M <= 256 && wgemm_wide() == 1 && p.K % 32 == 0) {
    const dim3 gw((p.N + 255) / 256);
    if (nt) wgemm_wide_kernel<true><<<gw, 512, 0, st>>>(p);
    else wgemm_wide_kernel<false><<<gw, 512, 0, st>>>(p);
    return;
  }
  switch (wmr) {
    case 1: if (nt) wgemm_kernel<1, true><<<grid, 512, 0, st>>>(p); else wgemm_kernel<1><<<grid, 512, 0, st>>>(p); break;
    case 2: if (nt) wgemm_kernel<2, true><<<grid, 512, 0, st>>>(p); else wgemm_kernel<2><<<grid, 512, 0, st>>>(p); break;
    default: if (nt) wgemm_kernel<4, true><<<grid, 512, 0, st>>>(p); else wgemm_kernel<4><<<grid, 512, 0, st>>>(p); break;
  }
}

}  // namespace akap
