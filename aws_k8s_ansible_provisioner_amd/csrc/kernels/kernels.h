// Host-visible launchers of the gfx950 kernels.  Pure HIP: no torch headers here,
// so every .hip translation unit compiles in seconds; torch glue lives in ops.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace akap {

// Ints per in-launch ticket counter: each counter on its own 128-B L2 line.  Atomics (and the
// relaxed polls of a spinning combine) on one line serialise at one L2 channel -- 1024 row
// tickets packed 32 to a line cost the sampler ~18 us at B = 16 (tools/sample_bench.py, s5c).
constexpr int kCtrStride = 32;
// the shared GEMM counter array (ops.gemm_counters): its size and the combine-timeout flag
constexpr int kCtrInts = 1 << 18;
constexpr int kCtrErr = kCtrInts - 1;


constexpr int kDecodeMaxPart = 8192;

// ---- norm.hip ----
void launch_rmsnorm(void* out, const void* x, const void* w, int rows, int d, int x_stride,
                    int out_stride, float eps, hipStream_t s);
void launch_fused_add_rmsnorm(void* out, void* residual, const void* x, const void* w, int rows,
                              int d, int x_stride, int out_stride, float eps, hipStream_t s);

// ---- rope_cache.hip ----
void launch_qk_norm_rope_cache(const void* qkv, int qkv_stride, void* q_out, void* k_cache,
                               void* v_cache, const int64_t* positions, const int64_t* slots,
                               const float* cos_sin, const void* q_w, const void* k_w, int T,
                               int Hq, int Hkv, int D, int BS, float eps, int apply_rope,
                               hipStream_t s, int kv_fp8 = 0, int v_per_token = 0,
                               void* v_tail = nullptr, const int* tail_slot = nullptr,
                               int num_decode = 0, int q_rows = -1);
void launch_reshape_and_cache(const void* k, const void* v, void* k_cache, void* v_cache,
                              const int64_t* slots, int T, int Hkv, int D, int BS, hipStream_t s,
                              int kv_fp8 = 0);

// ---- activation.hip ----
void launch_silu_and_mul(void* out, const void* in, long T, int F, int in_stride, hipStream_t s);

// ---- attention.hip ----
struct AttnParams {
  const __bf16* q;        // [T, Hq, D]
  const void* k_cache;    // [NB, Hkv, BS, D]        bf16, or fp8 bytes when kv_fp8
  const void* v_cache;    // [NB, Hkv, BS/8, D, 8]
  __bf16* out;            // [T, Hq, D]
  const int* block_tables;  // [B, bt_stride]
  int bt_stride;
  const int* seq_lens;  // [B] kv length incl. the new tokens
  const int* q_start;   // [B+1] cumulative query tokens (nullptr for pure decode)
  int Hq, Hkv, G, BS;
  float scale_log2;
  // prefill tiling (host-built): per 64-row tile its sequence and first flattened row
  const int* tile_seq;
  const int* tile_row;
  // decode split-KV (part_size <= kDecodeMaxPart: 64 wave steps of 128 tokens, one cache
  // block id per step held in a VGPR lane)
  int num_parts, part_size;
  float* part_m;  // [B, Hkv, parts, G]
  float* part_l;
  float* part_o;  // [B, Hkv, parts, G, D]
  int flags;      // reserved (0)
  int kv_fp8;     // caches hold OCP e4m3fn bytes (scale 1) instead of bf16
  // fused decode (qkv != nullptr): the kernel itself applies per-head q/k RMSNorm + RoPE to
  // the raw QKV projection row and writes the new token's K/V into the paged cache
  const __bf16* qkv;      // [B, qkv_stride]: q heads | k heads | v heads
  int qkv_stride;
  const int64_t* positions;  // [B]
  const int64_t* slots;      // [B] (-1: no write)
  const float* cos_sin;      // [max_pos, D] = cos | sin
  const __bf16* q_w;         // [D] or nullptr
  const __bf16* k_w;
  float eps;
  // V tail (bf16 caches; nullptr = off): per sequence slot, its current partial 8-token V
  // group token-major [slots, Hkv, 8, D] -- decode writes one 256-B row per token there and
  // the whole [D][8] group into the cache only when the group completes (16 full lines per
  // 8 tokens instead of 16 partial lines per token); decode readers take a partial group
  // from the tail.  tail_slot: per batch row (decode) / token (writer), -1 = no tail.
  __bf16* v_tail;
  const int* tail_slot;
  // prefill online softmax: a row's running max moves (and the O / l accumulators are
  // rescaled) only when the tile's max exceeds it by more than this many log2 units (0 =
  // every increase); set by launch_paged_attn_prefill (AKAP_FA_RESCALE_T, default 8)
  float rescale_t;
  // fused decode with the V tail: the new token's K / V cache and tail stores are issued at
  // the end of the work item from the LDS images instead of in the prologue (set by
  // launch_paged_attn_decode: AKAP_DECODE_DEFER_KV, default 1)
  int defer_kv;
};
// tile_rows: 128 -> flash-style LDS-tiled kernel (4 waves), 256 -> its 8-wave form (bf16 KV)
void launch_paged_attn_prefill(const AttnParams& p, int num_tiles, int tile_rows, hipStream_t s);
void launch_paged_attn_decode(const AttnParams& p, int num_seqs, hipStream_t s);

// ---- gemm.hip ----
int gemm_splitk_choice(int M, int N, int K);
// counters: zero-initialised int32 per-tile tickets (>= tiles) -> split-K partials are
// combined inside the launch by the last-arriving slice; nullptr -> separate reduce pass
void launch_gemm_bf16(const void* X, const void* W, void* Y, float* ws, int M, int N, int K,
                      int ldx, int ldw, int ldy, int splitk, hipStream_t st,
                      int* counters = nullptr);

// ---- dgemm.hip ----
// Fused decode GEMM: A-operand prologue (PRO_*) folded into the MFMA GEMM's staging, and an
// epilogue (EPI_*) doing a decode layer's residual add + next-norm elementwise half, or SwiGLU.
// Split-K partials (+ per-row sums of squares) are reduced by a second pass with the same epilogue.
enum { PRO_PLAIN = 0, PRO_ADDNORM = 1, PRO_SILU = 2 };
enum { EPI_STORE = 0, EPI_RESNORM = 1, EPI_SILU = 2 };
struct DGemmArgs {
  // bf16 tensors (void* so this header stays free of device types)
  const void* X;     // A source: [M, K] (PLAIN/ADDNORM) or [M, 2K] = [gate | up] (SILU)
  const void* R;     // ADDNORM: residual in [M, K] (row stride K)
  void* Rout;        // ADDNORM: residual out = X + R (must not alias R)
  const void* ln;    // ADDNORM: RMSNorm weight [K]
  const void* W;     // [N, K] (row stride ldw)
  void* Y;           // [M, N] (row stride ldy); EPI_RESNORM: residual in/out; EPI_SILU: [M, N/2]
  float* ws;         // split-K: fp32 [S, M, N] (+ [S, M] sums of squares for ADDNORM)
  const float* ss_in;  // PLAIN: optional per-row sum of squares -> rows scaled by rsqrt(ss/K+eps)
  float* ss_out;       // EPI_RESNORM: per-row sum of squares of the new residual (+= atomics)
  void* Aout;          // EPI_RESNORM: bf16(residual * ln_out) [M, N] dense
  const void* ln_out;  // EPI_RESNORM: next RMSNorm weight [N]
  int M, N, K, ldx, ldw, ldy, kps, epi;
  float eps;
  int bn;  // 0: register-ring kernel (dgemm.hip); 64 | 128: LDS-DMA ring kernel (gdgemm.hip)
  int ns;  // gdgemm ring depth: 0 = shallow (2 blocks/CU), >= 6 = deep ring (1 block/CU)
  int* counters;  // gdgemm split-K: zeroed per-tile tickets -> in-launch last-arriver combine
  int bm;         // gdgemm tile rows: 64 (default) | 128 (with bn = 128)
  int ntw;        // weight DMA policy: -1 default (gdgemm nt, kgemm not), 1 both nt, 0 neither
  int stag;       // 1: each workgroup walks its K range from a tile-dependent offset (wrapping)
};
// process default for DGemmArgs::ntw (AKAP_WEIGHT_NT, read once)
int weight_nt_default();
// process default for DGemmArgs::stag (AKAP_GEMM_STAGGER, read once)
int gemm_stagger_default();
// K-step at which tile (tm, tn) starts its walk of nk steps: workgroups that share an X panel
// (same tm) or a W panel (same tn) start at different steps, so the ones resident together do
// not request the same L2 lines at the same moment (hipBLASLt's "StaggerU")
__device__ __forceinline__ int gemm_stagger0(int stag, int tm, int tn, int nk) {
  return stag ? (tn + 3 * tm) % nk : 0;
}
bool dgemm_supported(int M, int N, int K, int splitk, int pf);
// split-K factors with a compiled reduce (1, 2, 4, 8, 16)
bool dgemm_splitk_ok(int splitk);
bool dgemm_epi_supported(int N, int epi, int splitk);
void launch_dgemm(const DGemmArgs& a, int pro, int splitk, int pf, hipStream_t st);
void launch_dgemm_reduce(const DGemmArgs& p, int pro, int splitk, hipStream_t st);
// gdgemm.hip: the same plain-prologue GEMM + epilogues with operands staged by global_load_lds
bool gdgemm_supported(int M, int N, int K, int splitk, int bn, int bm = 64);
// fp32 workspace floats a gdgemm split-K launch needs (tile-padded slabs)
long gdgemm_ws_floats(int M, int N, int splitk, int bn, int bm = 64);
void launch_gdgemm(const DGemmArgs& p, int splitk, hipStream_t st);
// kgemm.hip: BM (16 | 32) x 32 output tiles, K split over the workgroup's 4 waves (no global
// partials, no reduce launch); plain prologue, EPI_STORE / EPI_RESNORM, optional ss_in
bool kgemm_supported(int M, int N, int K, int bm);
void launch_kgemm(const DGemmArgs& p, int bm, hipStream_t st);

// ---- pgemm.hip: prefill / large-M GEMM Y = X . W^T, 256 x 256 tiles, optional expert groups
struct PGemmArgs {
  const void* X;    // bf16 [M, K] (row stride ldx); grouped: rows sorted by group
  const void* W;    // bf16 [N, K] dense, or [groups, N, K]
  void* Y;          // bf16 [M, N] (row stride ldy), or [M, N/2] with the SwiGLU epilogue
  const int* offs;  // grouped: [groups] cumulative row ends (device)
  int groups;       // 0 = dense
  int M, N, K, ldx, ldy;
  int stagger;      // unit body: workgroups start their K loops at decorrelated offsets
  int gm;           // raster: M tiles per block of the tile map (0 = 8)
};
bool pgemm_supported(int M, int N, int K);
void launch_pgemm(const PGemmArgs& p, int epi, hipStream_t st);
// decode-sized M: the same 256 x 256 body with K split over `splits` workgroups per tile and
// the slices combined in the launch (DGemmArgs epilogues: store | RESNORM | SILU, ss_in row
// scale).  Needs grid = tiles * splits <= the CU count (all slices resident); ws fp32
// pgemm_sk_ws_floats(); counters: 2 zeroed ints per tile (re-armed by the kernel), the error
// word at counters[65535].
bool pgemm_sk_supported(int M, int N, int K, int splits, int cus);
long pgemm_sk_ws_floats(int M, int N, int splits);
void launch_pgemm_sk(const DGemmArgs& p, int splits, hipStream_t st);

// ---- wgemm.hip: wide-row weight-streaming GEMM (LM head) Y[M,N] = X[M,K] . W[N,K]^T ----
struct WGemmArgs {
  const void* X;  // bf16 [M, K] (row stride ldx)
  const void* W;  // bf16 [N, K] (row stride ldw)
  void* Y;        // bf16 [M, N] (row stride ldy)
  int M, N, K, ldx, ldw, ldy;
};
bool wgemm_supported(int M, int N, int K, int ldx, int ldw, int ldy);
void launch_wgemm(const WGemmArgs& p, hipStream_t st);

// ---- sampling.hip ----
struct SampleParams {
  const void* logits;  // [B, V] (row stride ld), fp32 or bf16
  int ld, V;
  int is_bf16;
  const float* temperature;  // [B] (<=0 => greedy)
  const int* top_k;          // [B] (<=0 => off)
  const float* top_p;        // [B] (>=1 => off)
  const int64_t* seeds;      // [B]
  const int* steps;          // [B] per-request step counter mixed into the RNG
  int64_t* out_tokens;       // [B]
  float* out_logprobs;       // [B] log-prob of the sampled token (may be null)
  int greedy_logprobs;       // also compute log-probs for greedy rows (one extra pass)
};
// grid (sample_chunks(B, V) chunks, B rows); ws >= B * kMaxChunks * 32 bytes of partials,
// tickets[B] int32 zeroed once (each row's last chunk re-arms its ticket)
int sample_chunks(int B, int V, int wgs = 512);
// longest row the sampler covers: kMaxChunks chunks x kMaxTiles tiles x kTile elements
constexpr long kSampleMaxVocab = 64L * 64 * 2048;
long sample_ws_floats(int B);  // partial records + filter-pass states and histograms
// filtered = 0: the caller guarantees no row has top-k / top-p (their passes are not launched)
void launch_sample(const SampleParams& p, int B, void* ws, int* tickets, int filtered,
                   hipStream_t s);
// OpenAI/vLLM penalties on logits in place, for unique (row, token) entries:
// repetition (prompt + output tokens, divide positive / multiply negative logits),
// frequency * count and presence * [count > 0] (output tokens; count 0 = prompt-only)
void launch_apply_penalties(void* logits, int ld, int is_bf16, const int32_t* rows,
                            const int32_t* toks, const int32_t* counts, const float* presence,
                            const float* frequency, const float* repetition, int n,
                            hipStream_t s);
void launch_argmax(const void* logits, int ld, int V, int is_bf16, int64_t* out, int B,
                   hipStream_t s);

// ---- moe_dgemm.hip ----
// Grouped expert GEMM for MoE decode: 32|64-row x 128-col tiles, k-pipelined, optional
// activation-row gather and SwiGLU epilogue over gate/up-interleaved weight rows.
bool moe_dgemm_supported(int N, int K, int pf, int silu, int splitk);
void launch_moe_dgemm(const void* A, const void* W, void* Y, const int32_t* sorted_ids,
                      const int32_t* tile_expert, int max_tiles, int n_flat, int topk, int N,
                      int K, int lda, int ldy, int gather, int silu, int pf, int bm, int splitk,
                      float* partials, bool nt_weights, hipStream_t s);
// out[t] = sum_k w[t,k] * sum_z P[z, inv[t*K+k], :]  (split-K fp32 partials of the down GEMM)
void launch_moe_combine_split(const float* P, const float* wts, const int32_t* inv, void* out,
                              int T, int topk, int d, int S, int rows, hipStream_t s);

// ---- moe.hip ----
void launch_moe_topk_softmax(const void* logits, int ld, int E, int K, float* topk_w,
                             int32_t* topk_ids, int T, int renormalize, hipStream_t s);
// router GEMM (h [T, d] . W[E, d]^T, bf16-rounded logits) + softmax + top-k, E <= 16
bool moe_router_topk_supported(int E, int d);
void launch_moe_router_topk(const void* h, int ldh, const void* W, int d, int E, int K,
                            float* topk_w, int32_t* topk_ids, int T, int renormalize,
                            hipStream_t s);
void launch_moe_align(const int32_t* topk_ids, int n, int E, int block, int32_t* sorted_ids,
                      int32_t* expert_offsets, int32_t* num_padded, int32_t* inv,
                      int32_t* tile_expert, int max_tiles, hipStream_t s);
void launch_moe_gemm(const void* A, const void* W, void* Y, const int32_t* sorted_ids,
                     const int32_t* tile_expert, int max_tiles, int n_flat, int topk, int N,
                     int K, int lda, int gather, hipStream_t s);
void launch_moe_combine(const void* Y, const float* wts, const int32_t* inv, void* out, int T,
                        int topk, int d, hipStream_t s);

// ---- kv_transfer.hip ----
// The paged cache is `planes` planes (layer x {K,V}) of [NB, block_elems] bf16.
void launch_kv_gather(const void* cache, long plane_stride, int planes, int block_elems,
                      int cache_blocks, const int* block_ids, int nblk, void* out,
                      hipStream_t s);
void launch_kv_scatter(const void* in, void* cache, long plane_stride, int planes,
                       int block_elems, int cache_blocks, const int* block_ids, int nblk,
                       hipStream_t s);
// hipIpc pull: peer cache blocks -> own blocks, + V-tail fill of each request's partial
// last V group (see kv_transfer.hip)
struct KVPullArgs {
  // per-plane base addresses (device int64 tables [planes]): plane p of the source (a peer's
  // IPC-mapped cache, or this engine's own) and of this engine's cache; a cache may be several
  // allocations (layer-range segments), so planes are addressed through tables, not a stride
  const int64_t* src_planes;  // -> [NB_src, block_elems] bf16 each
  const int64_t* dst_planes;  // -> [NB, block_elems] bf16 each
  int planes, block_elems;
  const int* pairs;       // [nblk, 2]: (src block, dst block)
  int nblk;
  __bf16* tail;           // [layers, tail_slots, Hkv, 8, D] or nullptr
  const int* tail_jobs;   // [ntail, 4]: (src block, group, count 1..7, slot)
  int ntail, layers, tail_slots, Hkv, BS, D;
};
void launch_kv_pull(const KVPullArgs& a, hipStream_t s);

// ---- embedding.hip ----
void launch_embedding_prep(const int64_t* ids, const void* table, const void* ln, void* residual,
                           void* a_out, float* ss_out, float* zbuf, long zn, int T, int d,
                           int vocab_start, int vocab_end, hipStream_t s);
void launch_embedding(const int64_t* ids, const void* table, void* out, int T, int d,
                      int vocab_start, int vocab_end, hipStream_t s);

// ---- custom_allreduce.hip ----
struct CarArgs {
  __bf16* bufs[8];       // per-rank IPC-mapped buffers [4 * half_elems] (staging x2, result x2)
  uint32_t* sigs[8];     // per-rank IPC-mapped flag arrays
  uint32_t* counter;     // local per-block epoch counters
  uint32_t* err;         // local error flag (spin-wait timeout)
  int rank, world;
  size_t half_elems;     // capacity in elements of one staging half
  int blocks;            // grid of EVERY launch on this communicator (<= 128; see the header)
};
// Optional fused epilogue of the TP decode chain (the row-parallel O / down projection's
// partial sums are all-reduced, then): s = bf16(bf16(sum) + residual); residual = s;
// aout = bf16(s * ln[col]); ss[row] += s^2 -- the residual add + the elementwise half of the
// next RMSNorm, whose row scale the consumer GEMM applies (dgemm ss_in).  Rows are d wide.
struct CarEpi {
  __bf16* residual;  // [M, d] in/out
  const __bf16* ln;  // [d]
  __bf16* aout;      // [M, d]
  float* ss;         // [M] (+=; caller zeroes)
  int d;             // row width (multiple of 512: one wave's 64 x 8 elements share a row)
};
void launch_custom_allreduce(const CarArgs& a, const void* in, void* out, long n, int two_shot,
                             hipStream_t s, const CarEpi* epi = nullptr);
size_t custom_allreduce_signal_bytes();
// siblings on the same buffers / flags / epochs: rank-major all-gather of [rows, n] shards
// into [rows, world * n] (n % 8 == 0), and an in-place broadcast of `bytes` (% 16 == 0)
void launch_custom_allgather(const CarArgs& a, const void* in, void* out, long rows, int n,
                             hipStream_t s);
void launch_custom_broadcast(const CarArgs& a, void* buf, long bytes, int root, hipStream_t s);
// equal-segment all-to-all: in/out [world][seg_elems] bf16 (seg_elems % 8 == 0)
void launch_custom_alltoall(const CarArgs& a, const void* in, void* out, long seg_elems,
                            hipStream_t s);
struct CarMulti {  // test-only: every rank of a simulated group in one launch
  CarArgs args[8];
  const void* in[8];
  void* out[8];
  CarEpi epi[8];
  int use_epi;
  int warm;  // stress: pre-read peers' staging lines with plain loads (L1-warm consumer)
};
void launch_custom_allreduce_multi(const CarMulti& m, int world, long n, int two_shot,
                                   hipStream_t s);

// ---- prefetch.hip ----
struct PrefetchList {
  const void* ptr[8];
  long bytes[8];
  int n;
};
void launch_l2_prefetch(const PrefetchList& L, uint32_t* sink, hipStream_t s);
// host (pinned, device-mapped) -> device copy as a kernel on the stream
void launch_h2d_stage(const void* host_src, void* dst, long bytes, hipStream_t s);

}  // namespace akap
