// Loader / consumer ring GEMM for decode batches on gfx950:  Y[M,N] = X[M,K] . W[N,K]^T,
// M <= 256, wide N (Llama-3-8B gate|up: N = 28,672, K = 4,096), bf16 in, fp32 accumulate.
//
// Why (an experiment against the LDS-DMA decode tiles of gdgemm.hip): at M = 256 the decode
// GEMMs are bound by what each CU can pull from L2 / HBM (the whole X block plus its weight
// columns: ~3 MB per workgroup for gate|up), and the tuned tiles take in ~40 GB/s per CU while
// MI355X_MICROARCH.md ("ring-gemm") measures ~68 GB/s for a ring fed by dedicated loader
// waves.  Here one workgroup per column tile owns ALL rows (every weight byte crosses L2 -> CU
// once), and the 8 waves split by role:
//   waves 0-3 (loaders)   fill an NS-slot LDS ring, one 32-deep K step per slot, by LDS-DMA
//                         (global_load_lds, 16 B per lane); a step is published (FULL[s] += 1
//                         per loader wave) LAG steps after its issue, behind a counted vmcnt;
//                         a slot is refilled only after every consumer released it (FREE[s]);
//   waves 4-7 (consumers) each own 64 rows x BN columns: wait FULL, read the step's fragments,
//                         release the slot (FREE[s] += 1) once the reads retired, then MFMA
//                         16x16x32 (W fragment as A: the accumulator holds 4 consecutive
//                         output columns of one row per lane, stored as one 8-byte write).
// Counters live in the same LDS array as the ring (a second __shared__ object makes hipcc
// drain vmcnt), polled with s_sleep; every spin is bounded, and a run that would hang instead
// finishes with wrong values and raises p.err.
// LDS image: 64-B rows (32 bf16 of K), 16-B chunk c of row r stored at c ^ g[(r >> 2) & 3],
// g = {0, 2, 3, 1}: every ds_read_b128 lane group of a fragment read (rows {0-3, 12-15} at
// chunk c, rows {4-11} at c + 1) lands on 16 distinct 16-B bank slots.
#include "common.h"
#include "kernels.h"

namespace akap {

constexpr int RG_KS = 32;   // K per ring slot
constexpr int RG_ROWS = 256;
// ring slots and the steps a loader keeps in flight before publishing (NS > LAG + 1): as deep
// as 160 KiB of LDS allows (BN 64: 20 KB slots, BN 128: 24 KB)
template <int BN> struct RgRing { static constexpr int NS = BN == 64 ? 7 : 6, LAG = BN == 64 ? 4 : 3; };

// Ring counters are touched through inline asm: a compiler-visible LDS access in a wave with
// LDS-DMA in flight makes hipcc drain vmcnt(0) first (it cannot tell the DMA targets apart from
// the counter), which would serialise the ring to one step in flight.
__device__ __forceinline__ unsigned rg_lds(const int* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) int*)p;
}
__device__ __forceinline__ int rg_poll(const int* p) {
  int v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(rg_lds(p)) : "memory");
  return v;
}
__device__ __forceinline__ void rg_add(int* p) {
  asm volatile("ds_add_u32 %0, %1" ::"v"(rg_lds(p)), "v"(1) : "memory");
}

__device__ __forceinline__ int rg_g(int r) { return (0x1320 >> (((r >> 2) & 3) * 4)) & 3; }  // {0,2,3,1}

template <int BN>
__global__ __launch_bounds__(512, 1) void rgemm_kernel(RGemmArgs p) {
  constexpr int RG_NS = RgRing<BN>::NS, RG_LAG = RgRing<BN>::LAG;
  constexpr int SROWS = RG_ROWS + BN;          // rows per slot (X rows, then W rows)
  constexpr int SU = SROWS * 4;                // 16-B units per slot
  constexpr int PIECES = SROWS / 16;           // 1-KiB DMA pieces per slot
  static_assert(PIECES % 4 == 0, "pieces split evenly over the 4 loader waves");
  constexpr int PW = PIECES / 4;               // per loader wave
  constexpr int JN = BN / 16;
  __shared__ bf16x8 lds[RG_NS * SU + 8];       // + 2 x RG_NS counters (ints) at the end
  int* full = reinterpret_cast<int*>(lds + RG_NS * SU);
  int* freec = full + RG_NS;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = blockIdx.x * BN;
  const int nk = p.K / RG_KS;
  if (tid < 2 * RG_NS) full[tid] = 0;
  __syncthreads();

  if (w < 4) {
    // ---------------- loader ----------------
    const bf16* X = static_cast<const bf16*>(p.X);
    const bf16* W = static_cast<const bf16*>(p.W);
    const int lr = lane >> 2, pc = lane & 3;  // lane-linear destination: row, physical chunk
    const bf16* src[PW];
    int dst[PW];
#pragma unroll
    for (int e = 0; e < PW; ++e) {
      const int piece = w * PW + e;
      const int row = piece * 16 + lr;        // slot row
      const int ch = pc ^ rg_g(row);          // logical chunk this lane's 16 B hold
      if (row < RG_ROWS) {
        const int m = min(row, p.M - 1);      // rows past M re-read row M-1 (never stored)
        src[e] = X + (size_t)m * p.ldx + ch * 8;
      } else {
        src[e] = W + (size_t)(n0 + row - RG_ROWS) * p.ldw + ch * 8;
      }
      dst[e] = piece * 64;                    // 16-B units: 16 rows x 4 chunks
    }
    bool ok = true;
    for (int t = 0; t < nk + RG_LAG; ++t) {
      if (t < nk) {
        const int s = t % RG_NS, use = t / RG_NS;
        if (use > 0) {
          int spins = 0;
          while (rg_poll(freec + s) < use * 4) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1 << 22)) { ok = false; break; }
          }
        }
        bf16x8* slot = lds + s * SU;
#pragma unroll
        for (int e = 0; e < PW; ++e)
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)(src[e] + (size_t)t * RG_KS),
              (__attribute__((address_space(3))) void*)(slot + dst[e]), 16, 0, 0);
      }
      const int pub = t - RG_LAG;  // publish step pub: its DMAs retired
      if (pub >= 0) {
        if (t < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW * RG_LAG) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) rg_add(full + pub % RG_NS);
      }
    }
    if (!ok && lane == 0) __hip_atomic_fetch_or(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }

  // ---------------- consumer ----------------
  const int c = w - 4;                 // rows c*64 .. c*64+63
  const int fr = lane & 15, fg = lane >> 4;
  f32x4 acc[4][JN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bool ok = true;
  for (int t = 0; t < nk; ++t) {
    const int s = t % RG_NS, use = t / RG_NS;
    int spins = 0;
    while (rg_poll(full + s) < (use + 1) * 4) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1 << 22)) { ok = false; break; }
    }
    const bf16x8* slot = lds + s * SU;
    bf16x8 xf[4], wf[JN];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = c * 64 + i * 16 + fr;
      xf[i] = slot[row * 4 + (fg ^ rg_g(row))];
    }
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const int row = RG_ROWS + j * 16 + fr;
      wf[j] = slot[row * 4 + (fg ^ rg_g(row))];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) rg_add(freec + s);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }
  if (!ok && lane == 0) __hip_atomic_fetch_or(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // lane (fr, fg) of fragment (i, j): row c*64 + i*16 + fr, columns j*16 + fg*4 + 0..3
  bf16* Y = static_cast<bf16*>(p.Y);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = c * 64 + i * 16 + fr;
    if (row >= p.M) continue;
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r]);
      *reinterpret_cast<bf16x4*>(Y + (size_t)row * p.ldy + n0 + j * 16 + fg * 4) = o;
    }
  }
}

bool rgemm_supported(int M, int N, int K, int bn) {
  return M > 0 && M <= RG_ROWS && (bn == 64 || bn == 128) && N % bn == 0 && K % RG_KS == 0 &&
         K >= RG_KS;
}

void launch_rgemm(const RGemmArgs& p, int bn, hipStream_t st) {
  if (bn == 64) rgemm_kernel<64><<<p.N / 64, 512, 0, st>>>(p);
  else rgemm_kernel<128><<<p.N / 128, 512, 0, st>>>(p);
}

}  // namespace akap
