// Decode-GEMM ingress ceiling on one MI355X: how fast can the decode projections' operand tiles
// (X rows of the batch + W rows of the output columns, the bytes a GEMM workgroup must bring
// into its CU) be streamed into LDS with NO math, per shape, tile and ring depth, from cold
// (HBM) and warm (MALL-resident) weights?  If the streaming alone takes about as long as the
// GEMM kernel, the kernel sits at the ingress ceiling and only fewer bytes per CU (tiling) or
// overlap across launches can help; if it is much faster, the GEMM's pipeline is the loss.
//
// Each workgroup (WAVES x 64 threads) owns a BM x BN output tile, i.e. streams BM x K of X and
// BN x K of W in KST-deep stages through an NS-slot LDS ring by LDS-DMA (global_load_lds 16 B
// per lane), counted vmcnt + barrier per stage (the kgemm / pgemm discipline), and reads one
// 16-B LDS word per lane per stage so the data is consumed.  Grid: one workgroup per tile,
// a column tile's row tiles on one XCD (xcd_remap, as the GEMMs).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/ingress_probe tools/probes/ingress_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short bf16raw;

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

struct Args {
  const bf16raw* X;
  const bf16raw* W;
  int M, N, K, BM, BN, KST, NS;
  unsigned* out;
  int map;  // 0: xcd_remap (a column tile's row tiles on one XCD), 1: identity
  int op;   // 0: X and W rows, 1: X rows only (both halves from X), 2: W rows only
  int stag; // 1: each workgroup walks K from stage (blockIdx.x % stages), wrapping ("StaggerU")
};

__device__ __forceinline__ int tile_id(const Args& a, int nwg) {
  return a.map == 0 ? xcd_remap(blockIdx.x, nwg) : (int)blockIdx.x;
}
__device__ __forceinline__ const bf16raw* src_row(const Args& a, int row, int m0, int n0) {
  // op 1: the "W" rows re-read X rows (every operand byte from the shared 512 KB matrix);
  // op 2: the "X" rows read W rows of a disjoint range (nothing shared between row tiles)
  if (row < a.BM)
    return a.op == 2 ? a.W + (size_t)((n0 + row + a.BN) % a.N) * a.K : a.X + (size_t)(m0 + row) * a.K;
  return a.op == 1 ? a.X + (size_t)((m0 + row) % a.M) * a.K : a.W + (size_t)(n0 + row - a.BM) * a.K;
}

// LDS ring: NS slots of (BM + BN) rows x KST bf16.  DMA piece = 64 lanes x 16 B = 1 KiB.
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void k_ingress(Args a) {
  extern __shared__ u32x4 ring[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tiles_m = a.M / a.BM, tiles_n = a.N / a.BN;
  const int lt = tile_id(a, tiles_m * tiles_n);
  const int tn = lt / tiles_m, tm = lt % tiles_m;
  const int m0 = tm * a.BM, n0 = tn * a.BN;
  const int rows = a.BM + a.BN;
  const int cpr = a.KST / 8;                 // 16-B chunks per staged row
  const int units = rows * cpr;              // 16-B units per slot
  const int pieces = units / 64;             // 1 KiB DMA pieces per slot
  const int per_wave = (pieces + WAVES - 1) / WAVES;
  const int nst = a.K / a.KST;
  auto issue = [&](int st) {
    u32x4* slot = ring + (st % a.NS) * units;
    for (int i = 0; i < per_wave; ++i) {
      const int pc = w * per_wave + i;
      if (pc >= pieces) break;
      const int u = pc * 64 + lane;
      const int row = u / cpr, ch = u % cpr;
      const bf16raw* src = src_row(a, row, m0, n0) + (size_t)st * a.KST + ch * 8;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(slot + pc * 64),
                                       16, 0, 0);
    }
  };
  unsigned acc = 0;
  for (int s = 0; s < a.NS - 1 && s < nst; ++s) issue(s);
  for (int t = 0; t < nst; ++t) {
    // stages t+1 .. t+NS-2 may stay in flight: per_wave pieces per stage (uniform upper bound)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + a.NS - 1 < nst) issue(t + a.NS - 1);
    const u32x4* slot = ring + (t % a.NS) * units;
    acc ^= slot[(tid * 7) % units].x;
  }
  if (acc == 0x9e3779b9u) a.out[0] = acc;
}

// Variant with exact counted waits: compile-time pieces per wave (P) and depth (NS) so the
// vmcnt immediate is exact -- stages t+1..t+NS-2 stay in flight across the barrier.
// RD > 0: each wave also reads RD 16-B LDS words per lane per stage (a GEMM's fragment reads:
// pgemm's 8-wave tile reads 24 per 64-deep stage), to price the LDS traffic beside the DMA.
template <int WAVES, int P, int NS, int RD = 0>
__global__ __launch_bounds__(WAVES * 64, 1) void k_ingress_c(Args a) {
  extern __shared__ u32x4 ring[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tiles_m = a.M / a.BM, tiles_n = a.N / a.BN;
  const int lt = tile_id(a, tiles_m * tiles_n);
  const int tn = lt / tiles_m, tm = lt % tiles_m;
  const int m0 = tm * a.BM, n0 = tn * a.BN;
  const int cpr = a.KST / 8;
  const int units = (a.BM + a.BN) * cpr;
  const int nst = a.K / a.KST;
  const bf16raw* src[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int u = (w * P + i) * 64 + lane;
    const int row = u / cpr, ch = u % cpr;
    src[i] = src_row(a, row, m0, n0) + ch * 8;
  }
  const int st0 = a.stag ? (int)(blockIdx.x % nst) : 0;
  auto issue = [&](int st) {
    u32x4* slot = ring + (st % NS) * units;
    int ks = st + st0;
    if (ks >= nst) ks -= nst;
#pragma unroll
    for (int i = 0; i < P; ++i)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(src[i] + (size_t)ks * a.KST),
          (__attribute__((address_space(3))) void*)(slot + (w * P + i) * 64), 16, 0, 0);
  };
  unsigned acc = 0;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nst) issue(s);
  for (int t = 0; t < nst; ++t) {
    if (t + NS - 2 < nst) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P * (NS - 2)) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + NS - 1 < nst) issue(t + NS - 1);
    const u32x4* slot = ring + (t % NS) * units;
    if constexpr (RD > 0) {
      u32x4 v[RD];
#pragma unroll
      for (int i = 0; i < RD; ++i) v[i] = slot[(i * 64 * WAVES + tid * 5 + i) % units];
#pragma unroll
      for (int i = 0; i < RD; ++i) acc ^= v[i].x ^ v[i].w;
    } else {
      acc ^= slot[(tid * 7) % units].x;
    }
  }
  if (acc == 0x9e3779b9u) a.out[0] = acc;
}

// Register path: each thread loads its share of every stage straight into VGPRs
// (global_load_dwordx4), D stages in flight, no LDS.
template <int WAVES, int P, int D>
__global__ __launch_bounds__(WAVES * 64, 1) void k_ingress_reg(Args a) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tiles_m = a.M / a.BM, tiles_n = a.N / a.BN;
  const int lt = tile_id(a, tiles_m * tiles_n);
  const int tn = lt / tiles_m, tm = lt % tiles_m;
  const int m0 = tm * a.BM, n0 = tn * a.BN;
  const int cpr = a.KST / 8;
  const int nst = a.K / a.KST;
  const u32x4* src[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int u = (w * P + i) * 64 + lane;
    const int row = u / cpr, ch = u % cpr;
    src[i] = reinterpret_cast<const u32x4*>(src_row(a, row, m0, n0) + ch * 8);
  }
  u32x4 acc = {0, 0, 0, 0};
  u32x4 buf[D][P];
  const int st0 = a.stag ? (int)(blockIdx.x % nst) : 0;
  auto ko = [&](int st) { int k = st + st0; if (k >= nst) k -= nst; return (size_t)k * a.KST / 8; };
#pragma unroll
  for (int s = 0; s < D; ++s)
#pragma unroll
    for (int i = 0; i < P; ++i) buf[s][i] = s < nst ? src[i][ko(s)] : acc;
  for (int t = 0; t < nst; t += D) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
#pragma unroll
      for (int i = 0; i < P; ++i) acc ^= buf[s][i];
      if (t + s + D < nst) {
#pragma unroll
        for (int i = 0; i < P; ++i) buf[s][i] = src[i][ko(t + s + D)];
      }
    }
  }
  if ((acc.x ^ acc.y) == 0x9e3779b9u) a.out[0] = acc.x;
}

struct Shape {
  const char* name;
  int N, K;
};

int main(int argc, char** argv) {
  // optional filter: only configs whose CSV prefix "shape,tile,kst,ns,waves,path,map,op"
  // starts with argv[1] (one config per process for rocprofv3 --pmc passes)
  const char* filt = argc > 1 ? argv[1] : nullptr;
  const int reps = argc > 2 ? atoi(argv[2]) : 50;
  const int M = 256;
  Shape shapes[] = {{"qkv", 4096, 1024}, {"o", 1024, 2048}, {"gate_up", 6144, 1024},
                    {"down", 1024, 3072}};
  size_t wmax = (size_t)4096 * 4096;  // the largest prefill shape below (pf_l8b_o)
  for (auto& s : shapes) wmax = std::max(wmax, (size_t)s.N * s.K);
  bf16raw *X, *W;
  unsigned* out;
  void* flush;
  const size_t flush_bytes = 512ull << 20;
  const int MPF = 16384;  // prefill chunk rows (the pgemm / hipBLASLt shapes)
  CK(hipMalloc(&X, (size_t)MPF * 4096 * 2));
  CK(hipMalloc(&W, wmax * 2));
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&flush, flush_bytes));
  CK(hipMemset(X, 1, (size_t)MPF * 4096 * 2));
  CK(hipMemset(W, 1, wmax * 2));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("shape,tile,kst,ns,waves,path,map,op,stag,weights,us,bytes_per_cu_KB,GBps_per_cu,wgs\n");
  int MR = M;  // rows of the current shape set (decode 256, prefill MPF)
  auto run = [&](const char* nm, const Shape& s, int BM, int BN, int KST, int NS, int waves,
                 const char* path, int map, int op, int stag, auto launch) {
    char key[128];
    snprintf(key, sizeof key, "%s,%dx%d,%d,%d,%d,%s,%d,%d,%d", nm, BM, BN, KST, NS, waves,
             path, map, op, stag);
    if (filt && strncmp(key, filt, strlen(filt)) != 0) return;
    const int wgs = (MR / BM) * (s.N / BN);
    if ((size_t)s.N * s.K > wmax || (size_t)MR * s.K > (size_t)MPF * 4096) {
      fprintf(stderr, "skip %s: operands larger than the allocations\n", key);
      return;
    }
    const double per_cu = (double)(BM + BN) * s.K * 2;
    for (int cold = 0; cold < 2; ++cold) {
      float tot = 0.f;
      for (int r = 0; r < reps + 3; ++r) {
        if (cold) CK(hipMemsetAsync(flush, r & 0xff, flush_bytes, 0));
        CK(hipEventRecord(e0, 0));
        launch(wgs);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) tot += ms;
      }
      const double us = tot / reps * 1000.0;
      printf("%s,%s,%.2f,%.0f,%.1f,%d\n", key, cold ? "cold" : "warm", us, per_cu / 1024,
             per_cu / (us * 1e-6) / 1e9, wgs);
      fflush(stdout);
    }
  };
  for (auto& s : shapes) {
    struct T {
      int BM, BN, KST;
    };
    std::vector<T> tiles;
    if (s.N == 1024) tiles = {{32, 32, 256}, {64, 64, 128}};
    else if (s.N == 4096) tiles = {{64, 64, 128}, {128, 32, 256}};
    else tiles = {{64, 128, 128}, {64, 96, 128}};
    for (auto& t : tiles) {
      if (M % t.BM || s.N % t.BN || s.K % t.KST) continue;
      const int units = (t.BM + t.BN) * t.KST / 8;
      const int pieces = units / 64;
      for (int map = 0; map < 2; ++map)
        for (int op = 0; op < 3; ++op)
        for (int stag = 0; stag < 2; ++stag) {
          for (int NS : {4}) {
            const size_t lds = (size_t)NS * units * 16;
            if (lds > 160 * 1024) continue;
            Args a{X, W, M, s.N, s.K, t.BM, t.BN, t.KST, NS, out, map, op, stag};
            if (pieces % 4 == 0) {
              const int P = pieces / 4;
#define CASE(PP, NN)                                                                   \
  if (P == PP && NS == NN)                                                             \
    run(s.name, s, t.BM, t.BN, t.KST, NS, 4, "lds_counted", map, op, stag,             \
        [&](int wgs) { k_ingress_c<4, PP, NN><<<wgs, 256, lds, 0>>>(a); });
              CASE(4, 4) CASE(8, 4) CASE(6, 4) CASE(5, 4) CASE(10, 4) CASE(12, 4)
#undef CASE
            }
          }
          if (pieces % 4 == 0) {
            const int P = pieces / 4;
            Args a{X, W, M, s.N, s.K, t.BM, t.BN, t.KST, 0, out, map, op, stag};
#define RCASE(PP, DD)                                                                    \
  if (P == PP)                                                                           \
    run(s.name, s, t.BM, t.BN, t.KST, DD, 4, "reg", map, op, stag,                       \
        [&](int wgs) { k_ingress_reg<4, PP, DD><<<wgs, 256, 0, 0>>>(a); });
            RCASE(4, 2) RCASE(8, 2) RCASE(6, 2) RCASE(5, 2) RCASE(10, 2) RCASE(12, 2)
#undef RCASE
          }
        }
    }
  }
  // Prefill GEMM tiles (round 6, the pgemm-vs-hipBLASLt question): 256 x 256 output tiles at
  // M = 16384, the operand stream of one workgroup per tile (X 256 rows + W 256 rows, all K),
  // 64 KiB per 64-deep k-step.  Qwen3 o (N 1024, K 2048) is exactly 256 tiles (one per CU):
  // hipBLASLt runs it at 1.67 us per k-step (~10 TB/s of L2 -> CU), pgemm at ~2.6.
  MR = MPF;
  Shape pshapes[] = {{"pf_o", 1024, 2048}, {"pf_qkv", 4096, 1024}, {"pf_down", 1024, 3072},
                     {"pf_l8b_o", 4096, 4096}};
  for (auto& s : pshapes) {
    for (int stag = 0; stag < 2; ++stag) {
      Args a{X, W, MPF, s.N, s.K, 256, 256, 32, 4, out, 0, 0, stag};
      run(s.name, s, 256, 256, 32, 4, 8, "lds_counted", 0, 0, stag,
          [&](int wgs) { k_ingress_c<8, 4, 4><<<wgs, 512, 4 * 2048 * 16, 0>>>(a); });
      run(s.name, s, 256, 256, 32, 4, 4, "lds_counted", 0, 0, stag,
          [&](int wgs) { k_ingress_c<4, 8, 4><<<wgs, 256, 4 * 2048 * 16, 0>>>(a); });
      Args b2{X, W, MPF, s.N, s.K, 256, 256, 64, 2, out, 0, 0, stag};
      run(s.name, s, 256, 256, 64, 2, 8, "lds_counted", 0, 0, stag,
          [&](int wgs) { k_ingress_c<8, 8, 2><<<wgs, 512, 2 * 4096 * 16, 0>>>(b2); });
      if (!stag) {  // + the 8-wave GEMM's fragment reads (24 ds_read_b128 per lane per stage)
        run(s.name, s, 256, 256, 64, 2, 8, "lds_counted_rd24", 0, 0, stag,
            [&](int wgs) { k_ingress_c<8, 8, 2, 24><<<wgs, 512, 2 * 4096 * 16, 0>>>(b2); });
        run(s.name, s, 256, 256, 64, 2, 8, "lds_counted_rd12", 0, 0, stag,
            [&](int wgs) { k_ingress_c<8, 8, 2, 12><<<wgs, 512, 2 * 4096 * 16, 0>>>(b2); });
      }
      Args c{X, W, MPF, s.N, s.K, 256, 256, 32, 0, out, 0, 0, stag};
      run(s.name, s, 256, 256, 32, 2, 8, "reg", 0, 0, stag,
          [&](int wgs) { k_ingress_reg<8, 4, 2><<<wgs, 512, 0, 0>>>(c); });
    }
  }
  return 0;
}
