// torch custom-op registrations (namespace `akap`) for the gfx950 kernels.
//
// Every op launches on the caller's current HIP stream, allocates nothing and
// never synchronises, so all of them are hipGraph-capturable (engine decode path).
// PyTorch on ROCm names the GPU dispatch key "CUDA"; kernels are HIP/CDNA4 only.
#include <cstdlib>
#include <cstring>
#include <vector>
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "kernels/kernels.h"

namespace {

using at::Tensor;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

// KV caches are bf16, or uint8 holding OCP e4m3fn bytes (--kv-cache-dtype fp8)
int kv_fp8_of(const Tensor& k_cache, const Tensor& v_cache) {
  const bool f8 = k_cache.scalar_type() == at::kByte;
  TORCH_CHECK(f8 || k_cache.scalar_type() == at::kBFloat16, "KV cache must be bf16 or uint8 (fp8)");
  TORCH_CHECK(v_cache.scalar_type() == k_cache.scalar_type(), "K and V cache dtypes differ");
  return f8 ? 1 : 0;
}

#define CHECK_GPU(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_BF16(x) TORCH_CHECK((x).scalar_type() == at::kBFloat16, #x " must be bf16")
#define CHECK_LAST_CONTIG(x) TORCH_CHECK((x).stride(-1) == 1, #x " must have unit last stride")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")

void rmsnorm(Tensor out, Tensor x, Tensor w, double eps) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_LAST_CONTIG(x); CHECK_LAST_CONTIG(out);
  const int d = x.size(-1);
  TORCH_CHECK(d % 8 == 0, "hidden size must be a multiple of 8");
  const int rows = x.numel() / d;
  const c10::DeviceGuard g(x.device());
  akap::launch_rmsnorm(out.data_ptr(), x.data_ptr(), w.data_ptr(), rows, d,
                       x.dim() > 1 ? x.stride(-2) : d, out.dim() > 1 ? out.stride(-2) : d,
                       (float)eps, cur_stream());
}

void fused_add_rmsnorm(Tensor out, Tensor residual, Tensor x, Tensor w, double eps) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(residual); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_CONTIG(residual); CHECK_LAST_CONTIG(x); CHECK_LAST_CONTIG(out);
  const int d = x.size(-1);
  TORCH_CHECK(d % 8 == 0, "hidden size must be a multiple of 8");
  const int rows = x.numel() / d;
  const c10::DeviceGuard g(x.device());
  akap::launch_fused_add_rmsnorm(out.data_ptr(), residual.data_ptr(), x.data_ptr(), w.data_ptr(),
                                 rows, d, x.dim() > 1 ? x.stride(-2) : d,
                                 out.dim() > 1 ? out.stride(-2) : d, (float)eps, cur_stream());
}

void qk_norm_rope_cache(Tensor qkv, Tensor q_out, Tensor k_cache, Tensor v_cache,
                        Tensor positions, Tensor slots, Tensor cos_sin,
                        std::optional<Tensor> q_w, std::optional<Tensor> k_w, int64_t Hq,
                        int64_t Hkv, double eps, bool apply_rope, bool decode,
                        std::optional<Tensor> v_tail, std::optional<Tensor> tail_slot,
                        int64_t num_decode, int64_t q_rows) {
  CHECK_GPU(qkv); CHECK_BF16(qkv); CHECK_LAST_CONTIG(qkv); CHECK_CONTIG(q_out);
  TORCH_CHECK(q_rows >= -1 && q_rows <= qkv.size(0), "q_rows out of range");
  CHECK_CONTIG(k_cache); CHECK_CONTIG(v_cache);
  TORCH_CHECK(positions.scalar_type() == at::kLong && slots.scalar_type() == at::kLong,
              "positions/slots must be int64");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat, "cos_sin cache must be fp32");
  const int T = qkv.size(0);
  const int D = k_cache.size(3);
  const int BS = k_cache.size(2);
  TORCH_CHECK(D == 128, "head_dim must be 128");
  TORCH_CHECK(BS % 32 == 0, "block size must be a multiple of 32 (K cache chunk layout)");
  TORCH_CHECK(v_cache.dim() == 5 && v_cache.size(2) * 8 == BS && v_cache.size(3) == D &&
                  v_cache.size(4) == 8,
              "v_cache must be [NB,Hkv,BS/8,D,8]");
  TORCH_CHECK(qkv.size(1) >= (Hq + 2 * Hkv) * D, "qkv too narrow");
  TORCH_CHECK(positions.numel() >= T && slots.numel() >= T, "positions/slots too short");
  if (v_tail) {
    TORCH_CHECK(!decode, "the V tail is written by the span (prefill / mixed) role only");
    TORCH_CHECK(!kv_fp8_of(k_cache, v_cache), "the V tail needs a bf16 KV cache");
    TORCH_CHECK(tail_slot && tail_slot->scalar_type() == at::kInt && tail_slot->numel() >= T,
                "tail_slot: int32, one entry per token");
    TORCH_CHECK(v_tail->scalar_type() == at::kBFloat16 && v_tail->dim() == 4 &&
                    v_tail->size(1) == Hkv && v_tail->size(2) == 8 && v_tail->size(3) == D &&
                    v_tail->is_contiguous(),
                "v_tail must be contiguous bf16 [slots, Hkv, 8, 128]");
    TORCH_CHECK(num_decode >= 0 && num_decode <= T, "num_decode out of range");
  }
  const c10::DeviceGuard g(qkv.device());
  akap::launch_qk_norm_rope_cache(
      qkv.data_ptr(), qkv.stride(0), q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
      positions.data_ptr<int64_t>(), slots.data_ptr<int64_t>(), cos_sin.data_ptr<float>(),
      q_w ? q_w->data_ptr() : nullptr, k_w ? k_w->data_ptr() : nullptr, T, Hq, Hkv, D, BS,
      (float)eps, apply_rope ? 1 : 0, cur_stream(), kv_fp8_of(k_cache, v_cache), decode ? 1 : 0,
      v_tail ? v_tail->data_ptr() : nullptr, v_tail ? tail_slot->data_ptr<int>() : nullptr,
      (int)num_decode, (int)q_rows);
}

void reshape_and_cache(Tensor k, Tensor v, Tensor k_cache, Tensor v_cache, Tensor slots) {
  CHECK_GPU(k); CHECK_CONTIG(k); CHECK_CONTIG(v); CHECK_BF16(k); CHECK_BF16(v);
  const int T = k.size(0), Hkv = k.size(1), D = k.size(2);
  const int BS = k_cache.size(2);
  TORCH_CHECK(D == 128, "head_dim must be 128");
  TORCH_CHECK(BS % 32 == 0, "block size must be a multiple of 32 (K cache chunk layout)");
  const c10::DeviceGuard g(k.device());
  akap::launch_reshape_and_cache(k.data_ptr(), v.data_ptr(), k_cache.data_ptr(),
                                 v_cache.data_ptr(), slots.data_ptr<int64_t>(), T, Hkv, D, BS,
                                 cur_stream(), kv_fp8_of(k_cache, v_cache));
}

void silu_and_mul(Tensor out, Tensor x) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_LAST_CONTIG(x); CHECK_CONTIG(out);
  const int F = x.size(-1) / 2;
  TORCH_CHECK(F % 8 == 0, "ffn size must be a multiple of 8");
  const long T = x.numel() / x.size(-1);
  const c10::DeviceGuard g(x.device());
  akap::launch_silu_and_mul(out.data_ptr(), x.data_ptr(), T, F,
                            x.dim() > 1 ? x.stride(-2) : 2 * F, cur_stream());
}

// V tail arguments: v_tail [slots, Hkv, 8, D] bf16 (a bf16 cache only), tail_slot int32 with
// at least `rows` entries
static void set_v_tail(akap::AttnParams& p, const std::optional<Tensor>& v_tail,
                       const std::optional<Tensor>& tail_slot, int rows) {
  p.v_tail = nullptr;
  p.tail_slot = nullptr;
  if (!v_tail) return;
  TORCH_CHECK(tail_slot && tail_slot->scalar_type() == at::kInt && tail_slot->numel() >= rows,
              "tail_slot: int32 with one entry per row");
  TORCH_CHECK(v_tail->scalar_type() == at::kBFloat16 && v_tail->dim() == 4 &&
                  v_tail->size(1) == p.Hkv && v_tail->size(2) == 8 && v_tail->size(3) == 128 &&
                  v_tail->is_contiguous(),
              "v_tail must be contiguous bf16 [slots, Hkv, 8, 128]");
  TORCH_CHECK(!p.kv_fp8, "the V tail needs a bf16 KV cache");
  p.v_tail = (__bf16*)v_tail->data_ptr();
  p.tail_slot = tail_slot->data_ptr<int>();
}

akap::AttnParams attn_params(Tensor& out, Tensor& q, Tensor& k_cache, Tensor& v_cache,
                             Tensor& block_tables, Tensor& seq_lens, int64_t G, double scale) {
  CHECK_GPU(q); CHECK_BF16(q); CHECK_CONTIG(q); CHECK_CONTIG(out); CHECK_CONTIG(k_cache);
  CHECK_CONTIG(v_cache);
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && seq_lens.scalar_type() == at::kInt,
              "block_tables / seq_lens must be int32");
  TORCH_CHECK(block_tables.stride(1) == 1, "block_tables rows must be contiguous");
  akap::AttnParams p{};
  p.q = (const __bf16*)q.data_ptr();
  p.kv_fp8 = kv_fp8_of(k_cache, v_cache);
  p.k_cache = k_cache.data_ptr();
  p.v_cache = v_cache.data_ptr();
  p.out = (__bf16*)out.data_ptr();
  p.block_tables = block_tables.data_ptr<int>();
  p.bt_stride = block_tables.stride(0);
  p.seq_lens = seq_lens.data_ptr<int>();
  p.Hq = q.size(1);
  p.Hkv = k_cache.size(1);
  p.G = G;
  p.BS = k_cache.size(2);
  TORCH_CHECK(q.size(2) == 128 && k_cache.size(3) == 128, "attention kernels need head_dim 128");
  TORCH_CHECK(v_cache.dim() == 5 && v_cache.size(4) == 8, "v_cache must be [NB,Hkv,BS/8,D,8]");
  TORCH_CHECK(p.Hq == p.Hkv * G, "Hq must equal Hkv * G");
  TORCH_CHECK(p.BS % 32 == 0, "block size must be a multiple of 32 (K cache chunk layout)");
  p.scale_log2 = (float)(scale * 1.4426950408889634);
  return p;
}

void paged_attention_prefill(Tensor out, Tensor q, Tensor k_cache, Tensor v_cache,
                             Tensor block_tables, Tensor seq_lens, Tensor q_start,
                             Tensor tile_seq, Tensor tile_row, int64_t G, double scale,
                             int64_t tile_rows) {
  auto p = attn_params(out, q, k_cache, v_cache, block_tables, seq_lens, G, scale);
  TORCH_CHECK(tile_rows == 128 || tile_rows == 256, "tile_rows must be 128 or 256");
  TORCH_CHECK(tile_rows != 256 || k_cache.scalar_type() == at::kBFloat16,
              "tile_rows=256 needs a bf16 KV cache");
  // the flash-style kernel caches a sequence's block ids in LDS: <= 32768 keys
  TORCH_CHECK(block_tables.size(1) * k_cache.size(2) <= 32768,
              "prefill attention supports contexts up to 32768 tokens");
  TORCH_CHECK(q_start.scalar_type() == at::kInt && tile_seq.scalar_type() == at::kInt &&
                  tile_row.scalar_type() == at::kInt,
              "q_start/tile maps must be int32");
  p.q_start = q_start.data_ptr<int>();
  p.tile_seq = tile_seq.data_ptr<int>();
  p.tile_row = tile_row.data_ptr<int>();
  const c10::DeviceGuard g(q.device());
  akap::launch_paged_attn_prefill(p, tile_seq.numel(), (int)tile_rows, cur_stream());
}

// Prefill attention that reads its q rows raw from the QKV projection and applies the per-head
// q RMSNorm (q_w, optional) and NeoX RoPE itself (attention.hip, prefill kernel prologue): the
// standalone qk_norm_rope_cache pass then writes q only for the decode rows of a mixed step
// (q_rows = num_decode), saving the q write and re-read of every prefill token.
// The rotary row of a q token is its key index kv_len - q_len + i: the same invariant the
// kernel's causal mask relies on, and what the engine's positions hold for every prefill
// token.  `positions` is shape-checked and passed through but not read by the kernel.
void paged_attention_prefill_qprep(Tensor out, Tensor qkv, Tensor k_cache, Tensor v_cache,
                                   Tensor block_tables, Tensor seq_lens, Tensor q_start,
                                   Tensor tile_seq, Tensor tile_row, Tensor positions,
                                   Tensor cos_sin, std::optional<Tensor> q_w, int64_t G,
                                   double scale, double eps, int64_t tile_rows) {
  CHECK_GPU(qkv); CHECK_BF16(qkv); CHECK_LAST_CONTIG(qkv);
  TORCH_CHECK(positions.scalar_type() == at::kLong && positions.numel() >= qkv.size(0),
              "positions: int64, one per token");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() &&
                  cos_sin.size(-1) == 128,
              "cos_sin: contiguous fp32 [max_pos, 128]");
  TORCH_CHECK(qkv.size(0) == out.size(0), "qkv / out token counts differ");
  TORCH_CHECK(qkv.size(1) >= (out.size(1) + 2 * k_cache.size(1)) * 128, "qkv too narrow");
  TORCH_CHECK(qkv.stride(0) % 8 == 0 && (uintptr_t)qkv.data_ptr() % 16 == 0,
              "qkv rows must be 16-byte aligned");
  if (q_w) {
    CHECK_BF16(*q_w);
    TORCH_CHECK(q_w->is_contiguous() && q_w->numel() == 128, "q_w: contiguous bf16 [128]");
  }
  // `out` doubles as the q-shaped tensor for the shared parameter checks (same [T, Hq, D])
  auto p = attn_params(out, out, k_cache, v_cache, block_tables, seq_lens, G, scale);
  TORCH_CHECK(tile_rows == 128 || tile_rows == 256, "tile_rows must be 128 or 256");
  TORCH_CHECK(tile_rows != 256 || k_cache.scalar_type() == at::kBFloat16,
              "tile_rows=256 needs a bf16 KV cache");
  TORCH_CHECK(block_tables.size(1) * k_cache.size(2) <= 32768,
              "prefill attention supports contexts up to 32768 tokens");
  TORCH_CHECK(q_start.scalar_type() == at::kInt && tile_seq.scalar_type() == at::kInt &&
                  tile_row.scalar_type() == at::kInt,
              "q_start/tile maps must be int32");
  p.q = nullptr;
  p.qkv = (const __bf16*)qkv.data_ptr();
  p.qkv_stride = qkv.stride(0);
  p.positions = positions.data_ptr<int64_t>();
  p.cos_sin = cos_sin.data_ptr<float>();
  p.q_w = q_w ? (const __bf16*)q_w->data_ptr() : nullptr;
  p.eps = (float)eps;
  p.q_start = q_start.data_ptr<int>();
  p.tile_seq = tile_seq.data_ptr<int>();
  p.tile_row = tile_row.data_ptr<int>();
  const c10::DeviceGuard g(qkv.device());
  akap::launch_paged_attn_prefill(p, tile_seq.numel(), (int)tile_rows, cur_stream());
}

void paged_attention_decode(Tensor out, Tensor q, Tensor k_cache, Tensor v_cache,
                            Tensor block_tables, Tensor seq_lens, std::optional<Tensor> q_start,
                            Tensor part_m, Tensor part_l, Tensor part_o, int64_t num_parts,
                            int64_t part_size, int64_t G, double scale,
                            std::optional<Tensor> v_tail, std::optional<Tensor> tail_slot) {
  auto p = attn_params(out, q, k_cache, v_cache, block_tables, seq_lens, G, scale);
  TORCH_CHECK(G <= 16, "decode kernel supports up to 16 q heads per kv head");
  set_v_tail(p, v_tail, tail_slot, seq_lens.numel());
  TORCH_CHECK(part_size % 128 == 0 && part_size > 0 && part_size <= akap::kDecodeMaxPart,
              "part_size must be a multiple of 128, at most ", akap::kDecodeMaxPart);
  const int B = seq_lens.numel();
  p.q_start = q_start ? q_start->data_ptr<int>() : nullptr;
  p.num_parts = num_parts;
  p.part_size = part_size;
  if (num_parts > 1) {
    TORCH_CHECK(part_o.numel() >= (int64_t)B * p.Hkv * num_parts * G * 128,
                "part_o workspace too small");
    TORCH_CHECK(part_m.numel() >= (int64_t)B * p.Hkv * num_parts * G, "part_m too small");
    p.part_m = part_m.data_ptr<float>();
    p.part_l = part_l.data_ptr<float>();
    p.part_o = part_o.data_ptr<float>();
  }
  const c10::DeviceGuard g(q.device());
  akap::launch_paged_attn_decode(p, B, cur_stream());
}

// Decode attention fused with the per-head q/k RMSNorm + RoPE + new-token K/V cache write:
// reads the raw QKV projection rows, so the standalone qk_norm_rope_cache launch (and its
// q round trip) disappears from every decode layer.
void paged_attention_decode_fused(Tensor out, Tensor qkv, Tensor k_cache, Tensor v_cache,
                                  Tensor block_tables, Tensor seq_lens, Tensor positions,
                                  Tensor slots, Tensor cos_sin, std::optional<Tensor> q_w,
                                  std::optional<Tensor> k_w, Tensor part_m, Tensor part_l,
                                  Tensor part_o, int64_t num_parts, int64_t part_size, int64_t G,
                                  double scale, double eps, std::optional<Tensor> v_tail,
                                  std::optional<Tensor> tail_slot) {
  auto p = attn_params(out, out, k_cache, v_cache, block_tables, seq_lens, G, scale);
  set_v_tail(p, v_tail, tail_slot, seq_lens.numel());
  CHECK_GPU(qkv); CHECK_BF16(qkv); CHECK_LAST_CONTIG(qkv);
  TORCH_CHECK(G + 2 <= 16, "fused decode supports up to 14 q heads per kv head");
  TORCH_CHECK(part_size % 128 == 0 && part_size > 0 && part_size <= akap::kDecodeMaxPart,
              "part_size must be a multiple of 128, at most ", akap::kDecodeMaxPart);
  const int B = seq_lens.numel();
  TORCH_CHECK(qkv.size(0) >= B && qkv.size(1) >= (p.Hq + 2 * p.Hkv) * 128, "qkv shape");
  TORCH_CHECK(positions.scalar_type() == at::kLong && slots.scalar_type() == at::kLong,
              "positions / slots must be int64");
  TORCH_CHECK(positions.numel() >= B && slots.numel() >= B, "positions / slots too short");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.size(1) == 128, "cos_sin [P, 128]");
  p.q = nullptr;
  p.qkv = (const __bf16*)qkv.data_ptr();
  p.qkv_stride = qkv.stride(0);
  p.positions = positions.data_ptr<int64_t>();
  p.slots = slots.data_ptr<int64_t>();
  p.cos_sin = cos_sin.data_ptr<float>();
  p.q_w = q_w ? (const __bf16*)q_w->data_ptr() : nullptr;
  p.k_w = k_w ? (const __bf16*)k_w->data_ptr() : nullptr;
  p.eps = (float)eps;
  p.q_start = nullptr;
  p.num_parts = num_parts;
  p.part_size = part_size;
  if (num_parts > 1) {
    TORCH_CHECK(part_o.numel() >= (int64_t)B * p.Hkv * num_parts * G * 128,
                "part_o workspace too small");
    TORCH_CHECK(part_m.numel() >= (int64_t)B * p.Hkv * num_parts * G, "part_m too small");
    p.part_m = part_m.data_ptr<float>();
    p.part_l = part_l.data_ptr<float>();
    p.part_o = part_o.data_ptr<float>();
  }
  const c10::DeviceGuard g(qkv.device());
  akap::launch_paged_attn_decode(p, B, cur_stream());
}

void l2_prefetch(std::vector<Tensor> ts, Tensor sink) {
  TORCH_CHECK(ts.size() <= 8, "at most 8 tensors");
  akap::PrefetchList L{};
  for (size_t i = 0; i < ts.size(); ++i) {
    CHECK_GPU(ts[i]); CHECK_CONTIG(ts[i]);
    L.ptr[i] = ts[i].data_ptr();
    L.bytes[i] = (long)ts[i].numel() * ts[i].element_size();
  }
  L.n = ts.size();
  const c10::DeviceGuard g(sink.device());
  akap::launch_l2_prefetch(L, reinterpret_cast<uint32_t*>(sink.data_ptr<int>()), cur_stream());
}

int64_t gemm_splitk(int64_t M, int64_t N, int64_t K) {
  return akap::gemm_splitk_choice(M, N, K);
}

void gemm(Tensor out, Tensor x, Tensor w, Tensor ws, int64_t splitk,
          std::optional<Tensor> counters) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_LAST_CONTIG(x); CHECK_LAST_CONTIG(w); CHECK_LAST_CONTIG(out);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "gemm: 2-D tensors");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && out.size(0) == M && out.size(1) == N, "gemm: shape mismatch");
  TORCH_CHECK(K % 8 == 0 && N % 4 == 0, "gemm: K % 8, N % 4");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "gemm: 16-byte aligned rows");
  if (splitk > 1) {
    TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() >= splitk * M * N,
                "gemm: fp32 workspace of splitk*M*N");
  }
  int* cnt = nullptr;
  if (counters && splitk > 1) {
    TORCH_CHECK(counters->scalar_type() == at::kInt && counters->is_cuda(), "counters int32");
    TORCH_CHECK(counters->numel() >= (int64_t)((M + 63) / 64) * ((N + 63) / 64) * akap::kCtrStride,
                "counters: one L2 line (kCtrStride ints) per 64x64 tile");
    cnt = counters->data_ptr<int>();
  }
  const c10::DeviceGuard g(x.device());
  akap::launch_gemm_bf16(x.data_ptr(), w.data_ptr(), out.data_ptr(),
                         splitk > 1 ? ws.data_ptr<float>() : nullptr, M, N, K, x.stride(0),
                         w.stride(0), out.stride(0), splitk, cur_stream(), cnt);
}

// Fused decode GEMM: out = prologue(x, ...) @ w^T, then an epilogue.
// pro 0 plain (optional ss_in row scale), 1 residual-add + RMSNorm (r = residual in,
// rout = x + r out, ln = norm weight), 2 SiLU(gate) * up over x = [gate|up].
// epi 0 store, 1 residual/next-norm (out = residual in/out, aout = bf16(out * ln_out),
// ss_out += row sums of squares), 2 SwiGLU over gate/up-interleaved rows (out [M, N/2]).
// Compute units of a device (cached): the persistent / in-launch-combine GEMM grids must fit.
static int device_cus(int dev) {
  static int cached[16] = {0};
  if (dev < 0 || dev >= 16) dev = 0;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

void dgemm(Tensor out, Tensor x, Tensor w, Tensor ws, int64_t pro, int64_t splitk, int64_t pf,
           std::optional<Tensor> r, std::optional<Tensor> rout, std::optional<Tensor> ln,
           double eps, int64_t epi, std::optional<Tensor> ss_in, std::optional<Tensor> ss_out,
           std::optional<Tensor> aout, std::optional<Tensor> ln_out, int64_t bn, int64_t ns,
           std::optional<Tensor> counters, int64_t bm) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_LAST_CONTIG(x); CHECK_LAST_CONTIG(w); CHECK_LAST_CONTIG(out);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "dgemm: 2-D tensors");
  const int M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(pro >= 0 && pro <= 2, "dgemm: prologue 0|1|2");
  TORCH_CHECK(epi >= 0 && epi <= 2, "dgemm: epilogue 0|1|2");
  TORCH_CHECK(epi == 0 || pro == 0, "dgemm: epilogues 1|2 need the plain prologue");
  TORCH_CHECK(x.size(1) == (pro == akap::PRO_SILU ? 2 * K : K), "dgemm: x width");
  TORCH_CHECK(out.size(0) == M && out.size(1) == (epi == akap::EPI_SILU ? N / 2 : N),
              "dgemm: out shape");
  TORCH_CHECK(bn == 0 || pro == akap::PRO_PLAIN, "dgemm: the LDS-DMA variant has the plain prologue");
  TORCH_CHECK(bm == 64 || bn > 0, "dgemm: 128-row tiles are an LDS-DMA (bn > 0) variant");
  // bn == 256: the 256 x 256 pgemm body with an in-launch distributed split-K combine
  // (pgemm.hip pgemm_sk_kernel); the grid must fit the CUs (every slice resident)
  const bool sk = bn == 256;
  TORCH_CHECK(sk ? akap::pgemm_sk_supported(M, N, K, (int)splitk, device_cus(x.device().index()))
                 : bn > 0 ? akap::gdgemm_supported(M, N, K, splitk, bn, bm)
                          : akap::dgemm_supported(M, N, K, splitk, pf),
              "dgemm: unsupported M/N/K/splitk/pf/bn");
  TORCH_CHECK(!sk || splitk == 1 || counters.has_value(),
              "dgemm bn=256: split-K needs the counters (2 per tile)");
  // in-launch split-K combine: the LDS-DMA variants (bn > 0) and, with the plain prologue and
  // 2 | 4 | 8 slices, the register-ring kernel (64 x 64 tiles)
  const bool inlaunch = counters.has_value() && splitk > 1 &&
                        (bn > 0 || (pro == akap::PRO_PLAIN && (splitk == 2 || splitk == 4 ||
                                                               splitk == 8)));
  const int tile_n = bn > 0 ? (int)bn : 64, tile_m = bn > 0 ? (int)bm : 64;
  TORCH_CHECK(inlaunch ? (epi != akap::EPI_SILU || N % 32 == 0)
                       : akap::dgemm_epi_supported(N, epi, splitk),
              "dgemm: unsupported epilogue/N/splitk");
  TORCH_CHECK((int64_t)N * K * 2 >= (int64_t)M * 4, "dgemm: W smaller than M floats");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && out.stride(0) % 4 == 0,
              "dgemm: 16-byte aligned rows");
  if (splitk > 1) {
    const int64_t need = sk ? akap::pgemm_sk_ws_floats(M, N, (int)splitk)
                         : inlaunch ? akap::gdgemm_ws_floats(M, N, (int)splitk, tile_n, tile_m)
                                    : splitk * M * N + (pro == akap::PRO_ADDNORM ? splitk * M : 0);
    TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() >= need,
                "dgemm: fp32 workspace of splitk*M*N (+ splitk*M for the norm)");
    TORCH_CHECK(out.stride(0) == N || inlaunch || sk,
                "dgemm: split-K output must be dense (separate reduce pass)");
  }
  akap::DGemmArgs a{};
  a.ntw = akap::weight_nt_default();
  a.stag = akap::gemm_stagger_default();
  a.X = x.data_ptr();
  a.W = w.data_ptr();
  a.Y = out.data_ptr();
  a.ws = splitk > 1 ? ws.data_ptr<float>() : nullptr;
  a.M = M; a.N = N; a.K = K;
  a.ldx = x.stride(0); a.ldw = w.stride(0); a.ldy = out.stride(0);
  a.eps = (float)eps;
  a.epi = (int)epi;
  a.bn = (int)bn;
  a.ns = (int)ns;
  a.bm = (int)bm;
  if (inlaunch || (sk && counters && splitk > 1)) {
    // in-launch split-K combine: one zeroed int32 ticket per output tile
    TORCH_CHECK(counters->scalar_type() == at::kInt && counters->is_cuda() &&
                    counters->numel() >= (sk ? (int64_t)akap::kCtrInts
                                             : (int64_t)((M + tile_m - 1) / tile_m) *
                                                   ((N + tile_n - 1) / tile_n) * akap::kCtrStride),
                "dgemm: counters int32, one L2 line per output tile (bn=256: the kCtrInts array)");
    a.counters = counters->data_ptr<int>();
  }
  if (pro == akap::PRO_ADDNORM) {
    TORCH_CHECK(r && rout && ln, "dgemm addnorm: residual, residual-out and norm weight");
    CHECK_BF16(*r); CHECK_BF16(*rout); CHECK_BF16(*ln);
    CHECK_CONTIG(*r); CHECK_CONTIG(*rout); CHECK_CONTIG(*ln);
    TORCH_CHECK(r->numel() == (int64_t)M * K && rout->numel() == (int64_t)M * K &&
                ln->numel() == K, "dgemm addnorm: residual [M, K], norm weight [K]");
    TORCH_CHECK(r->data_ptr() != rout->data_ptr(), "dgemm addnorm: rout must not alias r");
    a.R = r->data_ptr();
    a.Rout = rout->data_ptr();
    a.ln = ln->data_ptr();
  }
  if (pro == akap::PRO_PLAIN && ss_in) {
    TORCH_CHECK(ss_in->scalar_type() == at::kFloat && ss_in->is_cuda() && ss_in->numel() >= M,
                "dgemm: ss_in fp32 [M]");
    a.ss_in = ss_in->data_ptr<float>();
  }
  if (epi == akap::EPI_RESNORM) {
    TORCH_CHECK(ss_out && aout && ln_out, "dgemm resnorm epilogue: ss_out, aout, ln_out");
    TORCH_CHECK(ss_out->scalar_type() == at::kFloat && ss_out->numel() >= M, "ss_out fp32 [M]");
    CHECK_BF16(*aout); CHECK_CONTIG(*aout); CHECK_BF16(*ln_out);
    TORCH_CHECK(aout->numel() == (int64_t)M * N && ln_out->numel() == N,
                "dgemm resnorm: aout [M, N], ln_out [N]");
    TORCH_CHECK(out.stride(0) == N, "dgemm resnorm: residual must be dense");
    a.ss_out = ss_out->data_ptr<float>();
    a.Aout = aout->data_ptr();
    a.ln_out = ln_out->data_ptr();
  }
  const c10::DeviceGuard g(x.device());
  if (sk) {
    akap::launch_pgemm_sk(a, (int)splitk, cur_stream());
    return;
  }
  akap::launch_dgemm(a, (int)pro, (int)splitk, (int)pf, cur_stream());
}

// Wide-row weight-streaming GEMM (LM head): out[M, N] = x[M, K] @ w[N, K]^T, one workgroup
// per column tile holding all (<= 256) rows, so the weights cross HBM -> CU once.
void wgemm(Tensor out, Tensor x, Tensor w) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_LAST_CONTIG(x); CHECK_LAST_CONTIG(w); CHECK_LAST_CONTIG(out);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "wgemm: 2-D tensors");
  const int M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(x.size(1) == K && out.size(0) == M && out.size(1) == N, "wgemm: shapes");
  TORCH_CHECK(akap::wgemm_supported(M, N, K, x.stride(0), w.stride(0), out.stride(0)),
              "wgemm: K % 64 == 0 and 16-byte aligned rows");
  akap::WGemmArgs a{x.data_ptr(), w.data_ptr(), out.data_ptr(), M, N, K,
                    (int)x.stride(0), (int)w.stride(0), (int)out.stride(0)};
  const c10::DeviceGuard g(x.device());
  akap::launch_wgemm(a, cur_stream());
}

// Narrow-output decode GEMM with the K split inside the workgroup (csrc/kernels/kgemm.hip):
// out = x @ w^T (rows scaled by rsqrt(ss_in / K + eps) when ss_in is given), epi 0 store,
// 1 residual/next-norm (out = residual in/out, aout = bf16(out * ln_out), ss_out += row sums).
void kgemm(Tensor out, Tensor x, Tensor w, int64_t bm, int64_t epi, double eps,
           std::optional<Tensor> ss_in, std::optional<Tensor> ss_out, std::optional<Tensor> aout,
           std::optional<Tensor> ln_out) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_LAST_CONTIG(x); CHECK_LAST_CONTIG(w); CHECK_LAST_CONTIG(out);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "kgemm: 2-D tensors");
  const int M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(x.size(1) == K && out.size(0) == M && out.size(1) == N, "kgemm: shapes");
  TORCH_CHECK(akap::kgemm_supported(M, N, K, (int)bm), "kgemm: bm 16|32, N % 32, K % 256");
  TORCH_CHECK(epi == 0 || epi == 1, "kgemm: epilogue 0|1");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && out.stride(0) % 4 == 0,
              "kgemm: aligned rows");
  akap::DGemmArgs a{};
  a.ntw = akap::weight_nt_default();
  a.stag = akap::gemm_stagger_default();
  a.X = x.data_ptr(); a.W = w.data_ptr(); a.Y = out.data_ptr();
  a.M = M; a.N = N; a.K = K;
  a.ldx = x.stride(0); a.ldw = w.stride(0); a.ldy = out.stride(0);
  a.eps = (float)eps;
  a.epi = (int)epi;
  if (ss_in) {
    TORCH_CHECK(ss_in->scalar_type() == at::kFloat && ss_in->numel() >= M, "ss_in fp32 [M]");
    a.ss_in = ss_in->data_ptr<float>();
  }
  if (epi == 1) {
    TORCH_CHECK(ss_out && aout && ln_out, "kgemm resnorm epilogue: ss_out, aout, ln_out");
    TORCH_CHECK(ss_out->scalar_type() == at::kFloat && ss_out->numel() >= M, "ss_out fp32 [M]");
    CHECK_BF16(*aout); CHECK_CONTIG(*aout); CHECK_BF16(*ln_out);
    TORCH_CHECK(aout->numel() == (int64_t)M * N && ln_out->numel() == N && out.stride(0) == N,
                "kgemm resnorm: aout [M, N], ln_out [N], dense residual");
    a.ss_out = ss_out->data_ptr<float>();
    a.Aout = aout->data_ptr();
    a.ln_out = ln_out->data_ptr();
  }
  const c10::DeviceGuard g(x.device());
  akap::launch_kgemm(a, (int)bm, cur_stream());
}

bool dgemm_ok(int64_t M, int64_t N, int64_t K, int64_t splitk, int64_t pf) {
  return akap::dgemm_supported(M, N, K, splitk, pf);
}

void sample(Tensor logits, Tensor temperature, Tensor top_k, Tensor top_p, Tensor seeds,
            Tensor steps, Tensor out_tokens, Tensor out_logprobs, bool greedy_logprobs,
            Tensor ws, Tensor tickets, bool filtered) {
  CHECK_GPU(logits);
  TORCH_CHECK(logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16,
              "sampler expects fp32 or bf16 logits");
  CHECK_LAST_CONTIG(logits);
  TORCH_CHECK(temperature.scalar_type() == at::kFloat && top_p.scalar_type() == at::kFloat,
              "temperature/top_p fp32");
  TORCH_CHECK(top_k.scalar_type() == at::kInt && steps.scalar_type() == at::kInt, "int32");
  TORCH_CHECK(seeds.scalar_type() == at::kLong && out_tokens.scalar_type() == at::kLong, "int64");
  const int B = logits.size(0);
  TORCH_CHECK(logits.size(1) >= 1 && logits.size(1) <= akap::kSampleMaxVocab,
              "sampler rows: 1 .. ", akap::kSampleMaxVocab, " logits");
  TORCH_CHECK(temperature.numel() >= B && top_k.numel() >= B && top_p.numel() >= B &&
                  seeds.numel() >= B && steps.numel() >= B && out_tokens.numel() >= B &&
                  (out_logprobs.numel() == 0 || out_logprobs.numel() >= B),
              "sampler: one parameter / output entry per row");
  akap::SampleParams p{};
  p.logits = logits.data_ptr();
  p.is_bf16 = logits.scalar_type() == at::kBFloat16;
  p.ld = logits.stride(0);
  p.V = logits.size(1);
  p.temperature = temperature.data_ptr<float>();
  p.top_k = top_k.data_ptr<int>();
  p.top_p = top_p.data_ptr<float>();
  p.seeds = seeds.data_ptr<int64_t>();
  p.steps = steps.data_ptr<int>();
  p.out_tokens = out_tokens.data_ptr<int64_t>();
  p.out_logprobs = out_logprobs.numel() ? out_logprobs.data_ptr<float>() : nullptr;
  p.greedy_logprobs = greedy_logprobs ? 1 : 0;
  // workspace: per-(row, chunk) 32-byte partial records + one ticket per row (ops.sample keeps
  // both persistent; the tickets are zeroed once and re-armed by each row's last chunk)
  CHECK_GPU(ws); CHECK_CONTIG(ws); CHECK_GPU(tickets); CHECK_CONTIG(tickets);
  TORCH_CHECK(ws.scalar_type() == at::kFloat && tickets.scalar_type() == at::kInt,
              "sampler workspace fp32, tickets int32");
  TORCH_CHECK(ws.numel() >= (int64_t)akap::sample_ws_floats(B),
              "sampler workspace too small (chunk records + filter-pass states / histograms)");
  TORCH_CHECK(tickets.numel() >= (int64_t)B * akap::kCtrStride,
              "one ticket per row, each on its own L2 line (kCtrStride ints)");
  const c10::DeviceGuard g(logits.device());
  akap::launch_sample(p, B, ws.data_ptr(), tickets.data_ptr<int>(), filtered ? 1 : 0,
                      cur_stream());
}

void apply_penalties(Tensor logits, Tensor rows, Tensor toks, Tensor counts, Tensor presence,
                     Tensor frequency, Tensor repetition) {
  CHECK_GPU(logits); CHECK_LAST_CONTIG(logits);
  TORCH_CHECK(logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16,
              "fp32 or bf16 logits");
  TORCH_CHECK(rows.scalar_type() == at::kInt && toks.scalar_type() == at::kInt &&
                  counts.scalar_type() == at::kInt, "rows/toks/counts int32");
  TORCH_CHECK(presence.scalar_type() == at::kFloat && frequency.scalar_type() == at::kFloat &&
                  repetition.scalar_type() == at::kFloat, "penalties fp32");
  const int n = rows.numel();
  TORCH_CHECK(toks.numel() == n && counts.numel() == n, "COO length mismatch");
  const c10::DeviceGuard g(logits.device());
  akap::launch_apply_penalties(logits.data_ptr(), logits.stride(0),
                               logits.scalar_type() == at::kBFloat16, rows.data_ptr<int>(),
                               toks.data_ptr<int>(), counts.data_ptr<int>(),
                               presence.data_ptr<float>(), frequency.data_ptr<float>(),
                               repetition.data_ptr<float>(), n, cur_stream());
}

void argmax(Tensor logits, Tensor out) {
  CHECK_GPU(logits); CHECK_LAST_CONTIG(logits);
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat,
              "argmax expects bf16/fp32");
  TORCH_CHECK(out.scalar_type() == at::kLong, "out int64");
  const c10::DeviceGuard g(logits.device());
  akap::launch_argmax(logits.data_ptr(), logits.stride(0), logits.size(1),
                      logits.scalar_type() == at::kBFloat16, out.data_ptr<int64_t>(),
                      logits.size(0), cur_stream());
}

void moe_topk_softmax(Tensor logits, Tensor topk_w, Tensor topk_ids, bool renorm) {
  CHECK_GPU(logits); CHECK_BF16(logits); CHECK_LAST_CONTIG(logits);
  TORCH_CHECK(logits.size(1) <= 256, "at most 256 experts");
  TORCH_CHECK(topk_w.size(1) >= 1 && topk_w.size(1) <= 8 && topk_w.size(1) <= logits.size(1),
              "top-k in 1..min(8, E)");
  TORCH_CHECK(topk_ids.sizes() == topk_w.sizes() && topk_w.size(0) == logits.size(0),
              "topk_w / topk_ids [T, K]");
  const c10::DeviceGuard g(logits.device());
  akap::launch_moe_topk_softmax(logits.data_ptr(), logits.stride(0), logits.size(1),
                                topk_w.size(1), topk_w.data_ptr<float>(),
                                topk_ids.data_ptr<int32_t>(), logits.size(0), renorm ? 1 : 0,
                                cur_stream());
}

void moe_router_topk(Tensor h, Tensor router, Tensor topk_w, Tensor topk_ids, bool renorm) {
  CHECK_GPU(h); CHECK_BF16(h); CHECK_LAST_CONTIG(h);
  CHECK_GPU(router); CHECK_BF16(router); CHECK_CONTIG(router);
  const int d = h.size(1), E = router.size(0);
  TORCH_CHECK(router.size(1) == d, "router shape");
  TORCH_CHECK(akap::moe_router_topk_supported(E, d), "fused router supports <= 16 experts, d % 8 == 0");
  TORCH_CHECK(topk_w.size(0) >= h.size(0) && topk_ids.size(0) >= h.size(0), "outputs too small");
  TORCH_CHECK(((uintptr_t)h.data_ptr() % 16) == 0 && h.stride(0) % 8 == 0, "h rows 16-B aligned");
  const c10::DeviceGuard g(h.device());
  akap::launch_moe_router_topk(h.data_ptr(), h.stride(0), router.data_ptr(), d, E, topk_w.size(1),
                               topk_w.data_ptr<float>(), topk_ids.data_ptr<int32_t>(), h.size(0),
                               renorm ? 1 : 0, cur_stream());
}

void moe_align(Tensor topk_ids, int64_t E, int64_t block, Tensor sorted_ids, Tensor offsets,
               Tensor num_padded, Tensor inv, Tensor tile_expert) {
  CHECK_GPU(topk_ids); CHECK_CONTIG(topk_ids);
  const int n = topk_ids.numel();
  TORCH_CHECK(sorted_ids.numel() >= n + E * (block - 1), "sorted_ids too small");
  TORCH_CHECK(inv.numel() == 0 || inv.numel() >= n, "inv too small");
  const int max_tiles = tile_expert.numel();
  TORCH_CHECK(max_tiles == 0 || (int64_t)max_tiles * block >= sorted_ids.numel(),
              "tile_expert must cover sorted_ids");
  const c10::DeviceGuard g(topk_ids.device());
  akap::launch_moe_align(topk_ids.data_ptr<int32_t>(), n, E, block,
                         sorted_ids.data_ptr<int32_t>(), offsets.data_ptr<int32_t>(),
                         num_padded.data_ptr<int32_t>(),
                         inv.numel() ? inv.data_ptr<int32_t>() : nullptr,
                         max_tiles ? tile_expert.data_ptr<int32_t>() : nullptr, max_tiles,
                         cur_stream());
}

void moe_gemm(Tensor out, Tensor a, Tensor w, Tensor sorted_ids, Tensor tile_expert,
              int64_t n_flat, int64_t topk, bool gather) {
  CHECK_GPU(a); CHECK_BF16(a); CHECK_BF16(w); CHECK_CONTIG(w); CHECK_CONTIG(out);
  CHECK_LAST_CONTIG(a);
  TORCH_CHECK(w.dim() == 3, "expert weights [E, N, K]");
  const int N = w.size(1), K = w.size(2);
  TORCH_CHECK(a.size(1) == K && out.size(1) == N, "moe_gemm shape mismatch");
  TORCH_CHECK(K % 8 == 0, "K % 8");
  const int max_tiles = tile_expert.numel();
  TORCH_CHECK(out.size(0) >= (int64_t)max_tiles * 64, "out rows must cover all tiles");
  if (!gather) TORCH_CHECK(a.size(0) >= (int64_t)max_tiles * 64, "a rows must cover all tiles");
  const c10::DeviceGuard g(a.device());
  akap::launch_moe_gemm(a.data_ptr(), w.data_ptr(), out.data_ptr(), sorted_ids.data_ptr<int32_t>(),
                        tile_expert.data_ptr<int32_t>(), max_tiles, n_flat, topk, N, K,
                        a.stride(0), gather ? 1 : 0, cur_stream());
}

// out: bf16 [rows, N] (or [rows, N/2] with silu); splitk > 1: out is an fp32 partials buffer
// [splitk, rows, N] consumed by moe_combine_split.
void moe_dgemm(Tensor out, Tensor a, Tensor w, Tensor sorted_ids, Tensor tile_expert,
               int64_t n_flat, int64_t topk, bool gather, bool silu, int64_t pf, int64_t bm,
               int64_t splitk) {
  CHECK_GPU(a); CHECK_BF16(a); CHECK_BF16(w); CHECK_CONTIG(w); CHECK_CONTIG(out);
  CHECK_LAST_CONTIG(a);
  TORCH_CHECK(w.dim() == 3, "expert weights [E, N, K]");
  const int N = w.size(1), K = w.size(2);
  TORCH_CHECK(a.size(1) == K, "moe_dgemm: a width != K");
  TORCH_CHECK(akap::moe_dgemm_supported(N, K, pf, silu, splitk), "moe_dgemm: unsupported N/K/pf/split");
  TORCH_CHECK(a.stride(0) % 8 == 0, "moe_dgemm: 16-byte aligned rows");
  TORCH_CHECK(sorted_ids.scalar_type() == at::kInt && tile_expert.scalar_type() == at::kInt,
              "moe_dgemm: int32 index tensors");
  TORCH_CHECK(bm == 32 || bm == 64, "moe_dgemm: tile rows 32 | 64");
  const int max_tiles = tile_expert.numel();
  const int64_t rows = (int64_t)max_tiles * bm;
  if (splitk > 1) {
    TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= splitk * rows * N,
                "moe_dgemm: fp32 partials [splitk, rows, N]");
  } else {
    CHECK_BF16(out);
    TORCH_CHECK(out.size(1) == (silu ? N / 2 : N), "moe_dgemm: out width");
    TORCH_CHECK(out.size(0) >= rows, "moe_dgemm: out rows must cover all tiles");
  }
  TORCH_CHECK(sorted_ids.numel() >= rows, "moe_dgemm: sorted_ids too short");
  if (!gather) TORCH_CHECK(a.size(0) >= rows, "moe_dgemm: a rows must cover all tiles");
  // Non-temporal expert-weight loads when each expert's weights are streamed by one row tile
  // (64-row tiles, <= 40 rows per expert on average): measured on MI355X, Mixtral T=128,
  // w13 345 -> 319 us, w2 (split 4) 226 -> 215 us; with 32-row tiles an expert's second tile
  // re-reads its weights and nt loses (bench/moe_gemm_micro.py, profiles/r2_moe_nt.log).
  // AKAP_MOE_NT=0|1 overrides.
  static const int nt_env = [] {
    const char* e = std::getenv("AKAP_MOE_NT");
    return e ? std::atoi(e) : -1;
  }();
  const bool ntw = nt_env >= 0 ? nt_env != 0 : (bm == 64 && n_flat <= 40 * w.size(0));
  const c10::DeviceGuard g(a.device());
  akap::launch_moe_dgemm(a.data_ptr(), w.data_ptr(), splitk > 1 ? nullptr : out.data_ptr(),
                         sorted_ids.data_ptr<int32_t>(), tile_expert.data_ptr<int32_t>(),
                         max_tiles, n_flat, topk, N, K, a.stride(0),
                         splitk > 1 ? N : out.stride(0), gather ? 1 : 0, silu ? 1 : 0, (int)pf,
                         (int)bm, (int)splitk, splitk > 1 ? out.data_ptr<float>() : nullptr, ntw,
                         cur_stream());
}

void moe_combine_split(Tensor partials, Tensor wts, Tensor inv, Tensor out, int64_t splitk,
                       int64_t rows) {
  CHECK_GPU(partials); CHECK_CONTIG(partials); CHECK_CONTIG(out); CHECK_BF16(out);
  TORCH_CHECK(partials.scalar_type() == at::kFloat, "partials fp32");
  TORCH_CHECK(wts.scalar_type() == at::kFloat && inv.scalar_type() == at::kInt, "dtypes");
  const int T = out.size(0), d = out.size(1), topk = wts.size(1);
  TORCH_CHECK(d % 8 == 0, "d % 8");
  TORCH_CHECK(partials.numel() >= splitk * rows * d, "partials [splitk, rows, d]");
  const c10::DeviceGuard g(out.device());
  akap::launch_moe_combine_split(partials.data_ptr<float>(), wts.data_ptr<float>(),
                                 inv.data_ptr<int32_t>(), out.data_ptr(), T, topk, d,
                                 (int)splitk, (int)rows, cur_stream());
}

void moe_combine(Tensor y, Tensor wts, Tensor inv, Tensor out) {
  CHECK_GPU(y); CHECK_BF16(y); CHECK_CONTIG(y); CHECK_CONTIG(out);
  TORCH_CHECK(wts.scalar_type() == at::kFloat && inv.scalar_type() == at::kInt, "dtypes");
  const int T = out.size(0), d = out.size(1), topk = wts.size(1);
  TORCH_CHECK(d % 8 == 0, "d % 8");
  const c10::DeviceGuard g(y.device());
  akap::launch_moe_combine(y.data_ptr(), wts.data_ptr<float>(), inv.data_ptr<int32_t>(),
                           out.data_ptr(), T, topk, d, cur_stream());
}

void kv_gather(Tensor cache, Tensor block_ids, Tensor out) {
  // cache: [planes, NB, ...block...]
  CHECK_GPU(cache); CHECK_CONTIG(cache); CHECK_CONTIG(out);
  const int planes = cache.size(0);
  const long plane_stride = cache.stride(0);
  const int block_elems = cache.stride(1);
  TORCH_CHECK(block_elems % 2048 == 0 || block_elems % 8 == 0, "block must be 16B multiple");
  TORCH_CHECK(out.numel() >= (int64_t)planes * block_ids.numel() * block_elems, "out too small");
  const c10::DeviceGuard g(cache.device());
  TORCH_CHECK(block_ids.is_cuda() && block_ids.scalar_type() == at::kInt, "int32 GPU block ids");
  akap::launch_kv_gather(cache.data_ptr(), plane_stride, planes, block_elems, cache.size(1),
                         block_ids.data_ptr<int>(), block_ids.numel(), out.data_ptr(),
                         cur_stream());
}

void kv_scatter(Tensor buf, Tensor cache, Tensor block_ids) {
  CHECK_GPU(cache); CHECK_CONTIG(cache); CHECK_CONTIG(buf);
  const int planes = cache.size(0);
  const c10::DeviceGuard g(cache.device());
  TORCH_CHECK(block_ids.is_cuda() && block_ids.scalar_type() == at::kInt, "int32 GPU block ids");
  TORCH_CHECK(buf.numel() >= (int64_t)planes * block_ids.numel() * cache.stride(1),
              "buf too small");
  akap::launch_kv_scatter(buf.data_ptr(), cache.data_ptr(), cache.stride(0), planes,
                          cache.stride(1), cache.size(1), block_ids.data_ptr<int>(),
                          block_ids.numel(), cur_stream());
}

// hipIpc KV pull (see kv_transfer.hip).  src_planes / dst_planes: int64 device tables of
// per-plane base addresses (a peer's planes as mapped by ipc_open -- or this engine's own for a
// tail-only fill -- and this engine's planes); every plane is [NB, block_elems] bf16 (an fp8
// cache moves as bf16 pairs).  Index ranges are validated by the caller
// (ops.kv_pull) before upload: the kernel trusts pairs / tail_jobs.
void kv_pull(Tensor src_planes, Tensor dst_planes, int64_t block_elems, Tensor pairs,
             std::optional<Tensor> tail, std::optional<Tensor> tail_jobs, int64_t Hkv,
             int64_t BS, int64_t D) {
  TORCH_CHECK(src_planes.scalar_type() == at::kLong && src_planes.is_cuda() &&
                  src_planes.is_contiguous() && dst_planes.scalar_type() == at::kLong &&
                  dst_planes.is_cuda() && dst_planes.is_contiguous() &&
                  src_planes.numel() == dst_planes.numel() && src_planes.numel() % 2 == 0,
              "plane tables: int64 [2L] on the device, same length");
  TORCH_CHECK(pairs.scalar_type() == at::kInt && pairs.is_cuda() && pairs.is_contiguous(),
              "pairs int32 [n, 2] on the device");
  TORCH_CHECK(pairs.numel() % 2 == 0, "pairs [n, 2]");
  akap::KVPullArgs a{};
  a.src_planes = src_planes.data_ptr<int64_t>();
  a.dst_planes = dst_planes.data_ptr<int64_t>();
  a.planes = src_planes.numel();
  a.block_elems = (int)block_elems;
  // bf16 cache: block = Hkv*BS*D; an fp8 (byte) cache is moved as bf16 pairs, block =
  // Hkv*BS*D/2 -- the copy jobs are dtype-agnostic 16-byte moves; V tails exist only for bf16
  const bool byte_cache = (int64_t)a.block_elems * 2 == Hkv * BS * D;
  TORCH_CHECK(a.block_elems % 8 == 0 && (a.block_elems == Hkv * BS * D || byte_cache),
              "block = Hkv*BS*D (bf16) or Hkv*BS*D/2 (fp8 bytes viewed as bf16)");
  a.pairs = pairs.data_ptr<int>();
  a.nblk = pairs.numel() / 2;
  a.Hkv = Hkv; a.BS = BS; a.D = D;
  a.layers = a.planes / 2;
  if (tail && tail_jobs && tail_jobs->numel()) {
    TORCH_CHECK(!byte_cache, "V-tail jobs need a bf16 cache");
    CHECK_CONTIG((*tail)); CHECK_BF16((*tail));
    TORCH_CHECK(tail->dim() == 5 && tail->size(0) == a.layers && tail->size(2) == Hkv &&
                tail->size(3) == 8 && tail->size(4) == D, "tail [L, slots, Hkv, 8, D]");
    TORCH_CHECK(tail_jobs->scalar_type() == at::kInt && tail_jobs->is_cuda() &&
                tail_jobs->is_contiguous() && tail_jobs->numel() % 4 == 0, "tail_jobs [m, 4]");
    TORCH_CHECK(BS % 8 == 0, "block size % 8");
    a.tail = reinterpret_cast<__bf16*>(tail->data_ptr());
    a.tail_slots = tail->size(1);
    a.tail_jobs = tail_jobs->data_ptr<int>();
    a.ntail = tail_jobs->numel() / 4;
  }
  const c10::DeviceGuard g(dst_planes.device());
  akap::launch_kv_pull(a, cur_stream());
}

// Prefill / large-M GEMM (pgemm.hip): out = x . w^T (epi 0) or silu(gate) * up over the
// [gate; up] halves of w (epi 2, out [M, N/2]).  offs (int32 [G], device) -> expert-grouped:
// rows of x sorted by group, w [G, N, K].
void pgemm(Tensor out, Tensor x, Tensor w, int64_t epi, std::optional<Tensor> offs) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_LAST_CONTIG(x); CHECK_CONTIG(w); CHECK_LAST_CONTIG(out);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2, "x, out must be 2-D");
  TORCH_CHECK(epi == akap::EPI_STORE || epi == akap::EPI_SILU, "pgemm epilogue: store | silu");
  akap::PGemmArgs a{};
  a.M = x.size(0);
  a.K = x.size(1);
  a.N = w.size(-2);
  TORCH_CHECK(w.size(-1) == a.K, "w [.., N, K] must match x [M, K]");
  TORCH_CHECK(akap::pgemm_supported(a.M, a.N, a.K), "pgemm: N % 256 == 0 and K % 64 == 0 needed");
  TORCH_CHECK(out.size(0) == a.M && out.size(1) == (epi == akap::EPI_SILU ? a.N / 2 : a.N),
              "out shape");
  if (offs) {
    TORCH_CHECK(w.dim() == 3 && offs->scalar_type() == at::kInt && offs->is_cuda() &&
                    offs->numel() == w.size(0),
                "grouped pgemm: w [G, N, K], offs int32 [G] on the device");
    a.offs = offs->data_ptr<int>();
    a.groups = offs->numel();
  } else {
    TORCH_CHECK(w.dim() == 2, "dense pgemm: w [N, K]");
  }
  a.X = x.data_ptr();
  a.W = w.data_ptr();
  a.Y = out.data_ptr();
  a.ldx = x.stride(0);
  a.ldy = out.stride(0);
  TORCH_CHECK(a.ldx % 8 == 0 && a.ldy % 4 == 0, "row strides must keep 16-B / 8-B alignment");
  // the DMA addresses X and one group's W through buffer descriptors with 32-bit offsets
  TORCH_CHECK((int64_t)a.M * a.ldx * 2 < (int64_t(1) << 31) &&
                  (int64_t)a.N * a.K * 2 < (int64_t(1) << 31),
              "pgemm: X and each weight matrix must stay below 2 GiB");
  const c10::DeviceGuard g(x.device());
  akap::launch_pgemm(a, (int)epi, cur_stream());
}

// dst (device) <- src (pinned host) by a kernel that reads the device mapping of the host
// buffer (no hipMemcpyAsync): the caller keeps src untouched until the stream passes it
void h2d_stage(Tensor dst, Tensor src) {
  CHECK_GPU(dst); CHECK_CONTIG(dst); CHECK_CONTIG(src);
  TORCH_CHECK(!src.is_cuda() && src.is_pinned(), "h2d_stage: src must be pinned host memory");
  TORCH_CHECK(src.nbytes() == dst.nbytes(), "h2d_stage: size mismatch");
  void* dev_src = nullptr;
  TORCH_CHECK(hipHostGetDevicePointer(&dev_src, src.data_ptr(), 0) == hipSuccess,
              "h2d_stage: the pinned buffer has no device mapping");
  const c10::DeviceGuard g(dst.device());
  akap::launch_h2d_stage(dev_src, dst.data_ptr(), (long)dst.nbytes(), cur_stream());
}

void embedding(Tensor ids, Tensor table, Tensor out, int64_t vocab_start, int64_t vocab_end) {
  CHECK_GPU(ids); CHECK_BF16(table); CHECK_CONTIG(table); CHECK_CONTIG(out);
  TORCH_CHECK(ids.scalar_type() == at::kLong, "ids int64");
  const int d = table.size(1);
  TORCH_CHECK(d % 8 == 0, "embedding dim multiple of 8");
  const c10::DeviceGuard g(ids.device());
  akap::launch_embedding(ids.data_ptr<int64_t>(), table.data_ptr(), out.data_ptr(), ids.numel(),
                         d, vocab_start, vocab_end, cur_stream());
}

void embedding_prep(Tensor ids, Tensor table, Tensor ln, Tensor residual, Tensor a_out,
                    Tensor ss_out, Tensor zbuf, int64_t vocab_start, int64_t vocab_end) {
  CHECK_GPU(ids); CHECK_BF16(table); CHECK_CONTIG(table); CHECK_BF16(ln); CHECK_CONTIG(ln);
  CHECK_BF16(residual); CHECK_CONTIG(residual); CHECK_BF16(a_out); CHECK_CONTIG(a_out);
  CHECK_CONTIG(ss_out); CHECK_CONTIG(zbuf);
  TORCH_CHECK(ids.scalar_type() == at::kLong, "ids int64");
  TORCH_CHECK(ss_out.scalar_type() == at::kFloat && zbuf.scalar_type() == at::kFloat,
              "ss_out / zbuf fp32");
  const int T = ids.numel(), d = table.size(1);
  TORCH_CHECK(d % 8 == 0 && ln.numel() == d, "embedding dim multiple of 8, ln of length d");
  TORCH_CHECK(residual.numel() == (int64_t)T * d && a_out.numel() == (int64_t)T * d &&
                  ss_out.numel() >= T,
              "residual / a_out [T, d], ss_out >= T");
  const c10::DeviceGuard g(ids.device());
  akap::launch_embedding_prep(ids.data_ptr<int64_t>(), table.data_ptr(), ln.data_ptr(),
                              residual.data_ptr(), a_out.data_ptr(), ss_out.data_ptr<float>(),
                              zbuf.data_ptr<float>(), zbuf.numel(), T, d, vocab_start, vocab_end,
                              cur_stream());
}

}  // namespace


// ---------------------------------------------------------------- custom all-reduce (K13)
// Per-communicator state lives here (C++), indexed by a small integer handle that the
// Python wrapper (parallel/custom_allreduce.py) keeps.  IPC handles are exchanged by the
// caller over torch.distributed.
namespace {
struct CarComm {
  int device = 0;
  akap::CarArgs args{};
  void* buf = nullptr;
  void* sig = nullptr;
  std::vector<void*> opened;
};
std::vector<CarComm*>& car_table() {
  static std::vector<CarComm*> t;
  return t;
}
CarComm* car_get(int64_t h) {
  auto& t = car_table();
  TORCH_CHECK(h >= 0 && h < (int64_t)t.size() && t[h] != nullptr, "bad custom all-reduce handle");
  return t[h];
}
#define HIP_OK(x)                                                                     \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    TORCH_CHECK(e_ == hipSuccess, #x " failed: ", hipGetErrorString(e_));             \
  } while (0)
}  // namespace

int64_t car_create(int64_t device, int64_t rank, int64_t world, int64_t max_elems,
                   int64_t blocks) {
  TORCH_CHECK(world >= 1 && world <= 8 && rank >= 0 && rank < world, "world must be 1..8");
  TORCH_CHECK(blocks >= 1 && blocks <= 128, "car blocks must be 1..128");
  TORCH_CHECK(max_elems % 8 == 0, "max_elems % 8");
  const c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (int)device));
  auto* c = new CarComm();
  c->device = (int)device;
  const size_t buf_bytes = (size_t)4 * max_elems * sizeof(uint16_t);
  const size_t sig_bytes = akap::custom_allreduce_signal_bytes();
  HIP_OK(hipExtMallocWithFlags(&c->buf, buf_bytes, hipDeviceMallocUncached));
  HIP_OK(hipExtMallocWithFlags(&c->sig, sig_bytes, hipDeviceMallocUncached));
  HIP_OK(hipMemset(c->sig, 0, sig_bytes));
  void* local = nullptr;
  HIP_OK(hipMalloc(&local, 4096));
  HIP_OK(hipMemset(local, 0, 4096));
  HIP_OK(hipDeviceSynchronize());
  c->args.counter = reinterpret_cast<uint32_t*>(local);
  c->args.err = reinterpret_cast<uint32_t*>(local) + 1023;
  c->args.rank = (int)rank;
  c->args.world = (int)world;
  c->args.half_elems = (size_t)max_elems;
  c->args.blocks = (int)blocks;
  for (int p = 0; p < 8; ++p) { c->args.bufs[p] = nullptr; c->args.sigs[p] = nullptr; }
  c->args.bufs[rank] = reinterpret_cast<__bf16*>(c->buf);
  c->args.sigs[rank] = reinterpret_cast<uint32_t*>(c->sig);
  car_table().push_back(c);
  return (int64_t)car_table().size() - 1;
}

Tensor car_ipc_handles(int64_t h) {
  CarComm* c = car_get(h);
  const c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, c->device));
  auto out = at::empty({2, (int64_t)sizeof(hipIpcMemHandle_t)}, at::kByte);
  hipIpcMemHandle_t hb, hs;
  HIP_OK(hipIpcGetMemHandle(&hb, c->buf));
  HIP_OK(hipIpcGetMemHandle(&hs, c->sig));
  std::memcpy(out.data_ptr<uint8_t>(), &hb, sizeof(hb));
  std::memcpy(out.data_ptr<uint8_t>() + sizeof(hb), &hs, sizeof(hs));
  return out;
}

void car_open(int64_t h, Tensor all_handles) {
  CarComm* c = car_get(h);
  TORCH_CHECK(all_handles.device().is_cpu() && all_handles.scalar_type() == at::kByte, "cpu uint8");
  TORCH_CHECK(all_handles.size(0) == c->args.world, "one handle pair per rank");
  const c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, c->device));
  auto hc = all_handles.contiguous();
  const uint8_t* base = hc.data_ptr<uint8_t>();
  const size_t hs = sizeof(hipIpcMemHandle_t);
  for (int p = 0; p < c->args.world; ++p) {
    if (p == c->args.rank) continue;
    hipIpcMemHandle_t hb, hg;
    std::memcpy(&hb, base + (size_t)p * 2 * hs, hs);
    std::memcpy(&hg, base + (size_t)p * 2 * hs + hs, hs);
    void* pb = nullptr;
    void* pg = nullptr;
    HIP_OK(hipIpcOpenMemHandle(&pb, hb, hipIpcMemLazyEnablePeerAccess));
    HIP_OK(hipIpcOpenMemHandle(&pg, hg, hipIpcMemLazyEnablePeerAccess));
    c->opened.push_back(pb);
    c->opened.push_back(pg);
    c->args.bufs[p] = reinterpret_cast<__bf16*>(pb);
    c->args.sigs[p] = reinterpret_cast<uint32_t*>(pg);
  }
}

// The IPC kernels move 16-byte vectors (bf16x8 loads / stores on the user tensors).
static void car_check_aligned(const Tensor& a, const Tensor& b) {
  TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0,
              "custom collective: tensors must be 16-byte aligned");
}

void car_all_reduce(int64_t h, Tensor inp, Tensor out, bool two_shot) {
  CarComm* c = car_get(h);
  CHECK_GPU(inp); CHECK_BF16(inp); CHECK_CONTIG(inp); CHECK_CONTIG(out); CHECK_BF16(out);
  TORCH_CHECK(inp.numel() == out.numel(), "size mismatch");
  TORCH_CHECK(inp.numel() % 8 == 0, "numel % 8");
  car_check_aligned(inp, out);
  TORCH_CHECK((size_t)inp.numel() <= c->args.half_elems, "message larger than the buffer");
  for (int p = 0; p < c->args.world; ++p)
    TORCH_CHECK(c->args.bufs[p] != nullptr, "peer buffers not opened (call car_open)");
  const c10::DeviceGuard g(inp.device());
  akap::launch_custom_allreduce(c->args, inp.data_ptr(), out.data_ptr(), inp.numel(),
                                two_shot ? 1 : 0, cur_stream());
}

static akap::CarEpi car_epi_of(Tensor& residual, Tensor& ln, Tensor& aout, Tensor& ss,
                               int64_t n) {
  CHECK_BF16(residual); CHECK_CONTIG(residual); CHECK_BF16(ln); CHECK_CONTIG(ln);
  CHECK_BF16(aout); CHECK_CONTIG(aout);
  const int64_t d = ln.numel();
  TORCH_CHECK(d % 512 == 0, "car resnorm: row width must be a multiple of 512");
  TORCH_CHECK(residual.numel() == n && aout.numel() == n && n % d == 0,
              "car resnorm: residual / aout [M, d] like the message");
  TORCH_CHECK(ss.scalar_type() == at::kFloat && ss.is_cuda() && ss.numel() >= n / d,
              "car resnorm: ss fp32 [M]");
  akap::CarEpi e{};
  e.residual = (__bf16*)residual.data_ptr();
  e.ln = (const __bf16*)ln.data_ptr();
  e.aout = (__bf16*)aout.data_ptr();
  e.ss = ss.data_ptr<float>();
  e.d = (int)d;
  return e;
}

// All-reduce of row-parallel partial sums fused with the decode chain's residual add and the
// elementwise half of the next RMSNorm (see CarEpi): residual += sum; aout = residual * ln;
// ss += row sums of residual^2.  `inp` is consumed (staged), nothing else is written.
void car_all_reduce_resnorm(int64_t h, Tensor inp, Tensor residual, Tensor ln, Tensor aout,
                            Tensor ss, bool two_shot) {
  CarComm* c = car_get(h);
  CHECK_GPU(inp); CHECK_BF16(inp); CHECK_CONTIG(inp);
  TORCH_CHECK((size_t)inp.numel() <= c->args.half_elems, "message larger than the buffer");
  for (int p = 0; p < c->args.world; ++p)
    TORCH_CHECK(c->args.bufs[p] != nullptr, "peer buffers not opened (call car_open)");
  const akap::CarEpi e = car_epi_of(residual, ln, aout, ss, inp.numel());
  car_check_aligned(inp, residual);
  car_check_aligned(ln, aout);
  const c10::DeviceGuard g(inp.device());
  akap::launch_custom_allreduce(c->args, inp.data_ptr(), nullptr, inp.numel(),
                                two_shot ? 1 : 0, cur_stream(), &e);
}

// Test hook: wire communicators created in THIS process (one per simulated rank, all on
// one GPU) to each other without IPC, so the kernel protocol can be exercised on 1 GPU.
void car_link_local(int64_t h, std::vector<int64_t> peers) {
  CarComm* c = car_get(h);
  TORCH_CHECK((int)peers.size() == c->args.world, "one handle per rank");
  for (int p = 0; p < c->args.world; ++p) {
    CarComm* o = car_get(peers[p]);
    c->args.bufs[p] = reinterpret_cast<__bf16*>(o->buf);
    c->args.sigs[p] = reinterpret_cast<uint32_t*>(o->sig);
  }
}

// Test hook: run the all-reduce of every simulated rank (communicators linked with
// car_link_local) in ONE grid, blockIdx.y = rank, so all ranks are co-resident regardless
// of how streams map to hardware queues.
void car_all_reduce_multi(std::vector<int64_t> hs, std::vector<Tensor> ins,
                          std::vector<Tensor> outs, bool two_shot,
                          std::optional<std::vector<Tensor>> epi, bool warm) {
  const int W = hs.size();
  TORCH_CHECK(W >= 1 && W <= 8 && (int)ins.size() == W && (int)outs.size() == W, "W ranks");
  akap::CarMulti m{};
  m.warm = warm ? 1 : 0;
  const int64_t n = ins[0].numel();
  for (int r = 0; r < W; ++r) {
    CarComm* c = car_get(hs[r]);
    TORCH_CHECK(c->args.world == W && c->args.rank == r, "handles must be ranks 0..W-1");
    CHECK_GPU(ins[r]); CHECK_BF16(ins[r]); CHECK_CONTIG(ins[r]); CHECK_CONTIG(outs[r]);
    TORCH_CHECK(ins[r].numel() == n && outs[r].numel() == n && n % 8 == 0, "sizes");
    TORCH_CHECK((size_t)n <= c->args.half_elems, "message larger than the buffer");
    m.args[r] = c->args;
    m.in[r] = ins[r].data_ptr();
    m.out[r] = outs[r].data_ptr();
    if (epi) {  // 4 tensors per rank: residual, ln, aout, ss
      TORCH_CHECK((int)epi->size() == 4 * W, "epi: residual, ln, aout, ss per rank");
      m.epi[r] = car_epi_of((*epi)[4 * r], (*epi)[4 * r + 1], (*epi)[4 * r + 2],
                            (*epi)[4 * r + 3], n);
      m.use_epi = 1;
    }
  }
  const c10::DeviceGuard g(ins[0].device());
  akap::launch_custom_allreduce_multi(m, W, n, two_shot ? 1 : 0, cur_stream());
}

int64_t car_error(int64_t h) {
  CarComm* c = car_get(h);
  const c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, c->device));
  uint32_t v = 0;
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(&v, c->args.err, sizeof(v), hipMemcpyDeviceToHost));
  return (int64_t)v;
}

// The communicator's device error word as a 1-element int32 tensor (no copy): a replayed
// decode graph enqueues an async copy of it to pinned host memory after its last collective,
// and the host checks it before the step's tokens are emitted (ModelRunner._err_probe).
Tensor car_error_word(int64_t h) {
  CarComm* c = car_get(h);
  return at::from_blob(c->args.err, {1},
                       at::TensorOptions().dtype(at::kInt).device(
                           c10::Device(c10::DeviceType::CUDA, c->device)));
}

// Rank-major all-gather of the vocab-parallel logits shard inp [R, n] -> out [R, W*n].
void car_all_gather(int64_t h, Tensor inp, Tensor out) {
  CarComm* c = car_get(h);
  CHECK_GPU(inp); CHECK_BF16(inp); CHECK_CONTIG(inp); CHECK_BF16(out); CHECK_CONTIG(out);
  const int64_t n = inp.size(-1);
  const int64_t rows = inp.numel() / n;
  TORCH_CHECK(n % 8 == 0, "shard width % 8");
  TORCH_CHECK(out.numel() == inp.numel() * c->args.world, "out [R, W*n]");
  car_check_aligned(inp, out);
  TORCH_CHECK((size_t)inp.numel() <= c->args.half_elems, "shard larger than the buffer");
  for (int p = 0; p < c->args.world; ++p)
    TORCH_CHECK(c->args.bufs[p] != nullptr, "peer buffers not opened (call car_open)");
  const c10::DeviceGuard g(inp.device());
  akap::launch_custom_allgather(c->args, inp.data_ptr(), out.data_ptr(), rows, (int)n,
                                cur_stream());
}

// Equal-segment all-to-all: inp/out [world * seg] bf16, segment d of inp goes to rank d and
// segment p of out comes from rank p.
void car_all_to_all(int64_t h, Tensor inp, Tensor out) {
  CarComm* c = car_get(h);
  CHECK_GPU(inp); CHECK_BF16(inp); CHECK_CONTIG(inp); CHECK_BF16(out); CHECK_CONTIG(out);
  const int64_t W = c->args.world;
  TORCH_CHECK(inp.numel() == out.numel() && inp.numel() % (W * 8) == 0,
              "all-to-all: inp/out [world * seg] with seg % 8 == 0");
  TORCH_CHECK((size_t)inp.numel() <= c->args.half_elems, "message larger than the buffer");
  TORCH_CHECK(inp.data_ptr() != out.data_ptr(), "all-to-all is out of place");
  car_check_aligned(inp, out);
  for (int p = 0; p < c->args.world; ++p)
    TORCH_CHECK(c->args.bufs[p] != nullptr, "peer buffers not opened (call car_open)");
  const c10::DeviceGuard g(inp.device());
  akap::launch_custom_alltoall(c->args, inp.data_ptr(), out.data_ptr(), inp.numel() / W,
                               cur_stream());
}

// In-place broadcast of buf (any dtype, nbytes % 16 == 0) from group rank `root`.
void car_broadcast(int64_t h, Tensor buf, int64_t root) {
  CarComm* c = car_get(h);
  CHECK_GPU(buf); CHECK_CONTIG(buf);
  const int64_t bytes = buf.numel() * buf.element_size();
  TORCH_CHECK(bytes % 16 == 0, "broadcast bytes % 16");
  car_check_aligned(buf, buf);
  TORCH_CHECK((size_t)bytes <= c->args.half_elems * 2, "message larger than the buffer");
  TORCH_CHECK(root >= 0 && root < c->args.world, "root rank");
  for (int p = 0; p < c->args.world; ++p)
    TORCH_CHECK(c->args.bufs[p] != nullptr, "peer buffers not opened (call car_open)");
  const c10::DeviceGuard g(buf.device());
  akap::launch_custom_broadcast(c->args, buf.data_ptr(), bytes, (int)root, cur_stream());
}

// ---------------------------------------------------------------- hipIpc of a whole tensor
// (the P/D KV pull): export -> [handle | offset of data_ptr in its allocation | bytes]
namespace {
std::vector<std::pair<int64_t, void*>>& ipc_opened() {
  static std::vector<std::pair<int64_t, void*>> t;
  return t;
}
}  // namespace

Tensor ipc_export(Tensor t) {
  CHECK_GPU(t);
  const c10::DeviceGuard g(t.device());
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  HIP_OK(hipMemGetAddressRange(&base, &size, t.data_ptr()));
  // ROCm 7.0.x runtimes (the one PyTorch bundles) hang in the PEER's hipIpcOpenMemHandle when
  // bit 31 of the allocation size is set (size mod 4 GiB >= 2 GiB; 7.2 maps them):
  // bench/ipc_import_repro.cpp, profiles/r6_ipc_import_sweep.md.  Refuse here instead of
  // letting the importer hang; KV segments are sized by models.transformer.ipc_safe_alloc_bytes
  int rt = 0;
  HIP_OK(hipRuntimeGetVersion(&rt));
  TORCH_CHECK(rt >= 70200000 || (size & (size_t(1) << 31)) == 0,
              "ipc_export: allocation of ", size, " bytes has bit 31 set; a peer's "
              "hipIpcOpenMemHandle of it hangs on this HIP runtime (", rt,
              "): pad it to a multiple of 4 GiB (ipc_safe_alloc_bytes)");
  hipIpcMemHandle_t hd;
  HIP_OK(hipIpcGetMemHandle(&hd, base));
  const int64_t off = (int64_t)((char*)t.data_ptr() - (char*)base);
  const int64_t nbytes = t.numel() * t.element_size();
  TORCH_CHECK(off >= 0 && (size_t)(off + nbytes) <= size, "tensor outside its allocation");
  auto out = at::empty({(int64_t)sizeof(hd) + 16}, at::kByte);
  std::memcpy(out.data_ptr<uint8_t>(), &hd, sizeof(hd));
  std::memcpy(out.data_ptr<uint8_t>() + sizeof(hd), &off, 8);
  std::memcpy(out.data_ptr<uint8_t>() + sizeof(hd) + 8, &nbytes, 8);
  return out;
}

// Map a peer's exported tensor; returns its device address (valid on `device` until
// ipc_close).  The same GPU (two processes) or a peer GPU over xGMI.
int64_t ipc_open(Tensor blob, int64_t device) {
  TORCH_CHECK(blob.device().is_cpu() && blob.scalar_type() == at::kByte &&
              blob.numel() == (int64_t)sizeof(hipIpcMemHandle_t) + 16, "ipc_export blob");
  const c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (int)device));
  auto b = blob.contiguous();
  hipIpcMemHandle_t hd;
  int64_t off = 0;
  std::memcpy(&hd, b.data_ptr<uint8_t>(), sizeof(hd));
  std::memcpy(&off, b.data_ptr<uint8_t>() + sizeof(hd), 8);
  void* p = nullptr;
  HIP_OK(hipIpcOpenMemHandle(&p, hd, hipIpcMemLazyEnablePeerAccess));
  const int64_t addr = (int64_t)((char*)p + off);
  ipc_opened().emplace_back(addr, p);
  return addr;
}

void ipc_close(int64_t addr) {
  auto& t = ipc_opened();
  for (size_t i = 0; i < t.size(); ++i)
    if (t[i].first == addr) {
      (void)hipIpcCloseMemHandle(t[i].second);
      t.erase(t.begin() + i);
      return;
    }
}

void car_destroy(int64_t h) {
  CarComm* c = car_get(h);
  const c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, c->device));
  (void)hipDeviceSynchronize();
  for (void* p : c->opened) (void)hipIpcCloseMemHandle(p);
  (void)hipFree(c->buf);
  (void)hipFree(c->sig);
  (void)hipFree(c->args.counter);
  delete c;
  car_table()[h] = nullptr;
}

TORCH_LIBRARY(akap, m) {
  m.def("rmsnorm(Tensor(a!) out, Tensor x, Tensor w, float eps) -> ()");
  m.def("fused_add_rmsnorm(Tensor(a!) out, Tensor(b!) residual, Tensor x, Tensor w, float eps) -> ()");
  m.def(
      "qk_norm_rope_cache(Tensor qkv, Tensor(a!) q_out, Tensor(b!) k_cache, Tensor(c!) v_cache, "
      "Tensor positions, Tensor slots, Tensor cos_sin, Tensor? q_w, Tensor? k_w, int Hq, int Hkv, "
      "float eps, bool apply_rope, bool decode=False, Tensor(d!)? v_tail=None, "
      "Tensor? tail_slot=None, int num_decode=0, int q_rows=-1) -> ()");
  m.def("reshape_and_cache(Tensor k, Tensor v, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor slots) -> ()");
  m.def("silu_and_mul(Tensor(a!) out, Tensor x) -> ()");
  m.def(
      "paged_attention_prefill(Tensor(a!) out, Tensor q, Tensor k_cache, Tensor v_cache, "
      "Tensor block_tables, Tensor seq_lens, Tensor q_start, Tensor tile_seq, Tensor tile_row, "
      "int G, float scale, int tile_rows=128) -> ()");
  m.def(
      "paged_attention_prefill_qprep(Tensor(a!) out, Tensor qkv, Tensor k_cache, Tensor v_cache, "
      "Tensor block_tables, Tensor seq_lens, Tensor q_start, Tensor tile_seq, Tensor tile_row, "
      "Tensor positions, Tensor cos_sin, Tensor? q_w, int G, float scale, float eps, "
      "int tile_rows=128) -> ()");
  m.def(
      "paged_attention_decode(Tensor(a!) out, Tensor q, Tensor k_cache, Tensor v_cache, "
      "Tensor block_tables, Tensor seq_lens, Tensor? q_start, Tensor(b!) part_m, Tensor(c!) part_l, "
      "Tensor(d!) part_o, int num_parts, int part_size, int G, float scale, "
      "Tensor? v_tail=None, Tensor? tail_slot=None) -> ()");
  m.def(
      "paged_attention_decode_fused(Tensor(a!) out, Tensor qkv, Tensor(b!) k_cache, "
      "Tensor(c!) v_cache, Tensor block_tables, Tensor seq_lens, Tensor positions, Tensor slots, "
      "Tensor cos_sin, Tensor? q_w, Tensor? k_w, Tensor(d!) part_m, Tensor(e!) part_l, "
      "Tensor(f!) part_o, int num_parts, int part_size, int G, float scale, float eps, "
      "Tensor(g!)? v_tail=None, Tensor? tail_slot=None) -> ()");
  m.def(
      "sample(Tensor logits, Tensor temperature, Tensor top_k, Tensor top_p, Tensor seeds, "
      "Tensor steps, Tensor(a!) out_tokens, Tensor(b!) out_logprobs, "
      "bool greedy_logprobs, Tensor(c!) ws, Tensor(d!) tickets, bool filtered=True) -> ()");
  m.def(
      "apply_penalties(Tensor(a!) logits, Tensor rows, Tensor toks, Tensor counts, "
      "Tensor presence, Tensor frequency, Tensor repetition) -> ()");
  m.def("argmax(Tensor logits, Tensor(a!) out) -> ()");
  m.def(
      "gemm(Tensor(a!) out, Tensor x, Tensor w, Tensor(b!) ws, int splitk, "
      "Tensor(c!)? counters=None) -> ()");
  m.def("gemm_splitk(int M, int N, int K) -> int");
  m.def(
      "dgemm(Tensor(a!) out, Tensor x, Tensor w, Tensor(b!) ws, int pro, int splitk, int pf, "
      "Tensor? r=None, Tensor(c!)? rout=None, Tensor? ln=None, float eps=1e-6, int epi=0, "
      "Tensor? ss_in=None, Tensor(d!)? ss_out=None, Tensor(e!)? aout=None, "
      "Tensor? ln_out=None, int bn=0, int ns=0, Tensor(f!)? counters=None, int bm=64) -> ()");
  m.def("wgemm(Tensor(a!) out, Tensor x, Tensor w) -> ()");
  m.def("pgemm(Tensor(a!) out, Tensor x, Tensor w, int epi=0, Tensor? offs=None) -> ()");
  m.def("kgemm(Tensor(a!) out, Tensor x, Tensor w, int bm, int epi, float eps, Tensor? ss_in, "
        "Tensor(b!)? ss_out, Tensor(c!)? aout, Tensor? ln_out) -> ()");
  m.def("dgemm_ok(int M, int N, int K, int splitk, int pf) -> bool");
  m.def("l2_prefetch(Tensor[] ts, Tensor(a!) sink) -> ()");
  m.def("car_create(int device, int rank, int world, int max_elems, int blocks=128) -> int");
  m.def("car_ipc_handles(int h) -> Tensor");
  m.def("car_open(int h, Tensor handles) -> ()");
  m.def("car_all_reduce(int h, Tensor inp, Tensor(a!) out, bool two_shot) -> ()");
  m.def("car_error(int h) -> int");
  m.def("car_error_word(int h) -> Tensor");
  m.def("car_link_local(int h, int[] peers) -> ()");
  m.def("car_all_reduce_multi(int[] hs, Tensor[] ins, Tensor(a!)[] outs, bool two_shot, "
        "Tensor(b!)[]? epi=None, bool warm=False) -> ()");
  m.def("car_all_reduce_resnorm(int h, Tensor inp, Tensor(a!) residual, Tensor ln, "
        "Tensor(b!) aout, Tensor(c!) ss, bool two_shot) -> ()");
  m.def("car_destroy(int h) -> ()");
  m.def("car_all_gather(int h, Tensor inp, Tensor(a!) out) -> ()");
  m.def("car_broadcast(int h, Tensor(a!) buf, int root) -> ()");
  m.def("car_all_to_all(int h, Tensor inp, Tensor(a!) out) -> ()");
  m.def("h2d_stage(Tensor(a!) dst, Tensor src) -> ()");
  m.def("ipc_export(Tensor t) -> Tensor");
  m.def("ipc_open(Tensor blob, int device) -> int");
  m.def("ipc_close(int addr) -> ()");
  m.def(
      "kv_pull(Tensor src_planes, Tensor dst_planes, int block_elems, Tensor pairs, "
      "Tensor(a!)? tail, Tensor? tail_jobs, int Hkv, int BS, int D) -> ()");
  m.def("moe_topk_softmax(Tensor logits, Tensor(a!) topk_w, Tensor(b!) topk_ids, bool renorm) -> ()");
  m.def("moe_router_topk(Tensor h, Tensor router, Tensor(a!) topk_w, Tensor(b!) topk_ids, bool renorm) -> ()");
  m.def(
      "moe_align(Tensor topk_ids, int E, int block, Tensor(a!) sorted_ids, Tensor(b!) offsets, "
      "Tensor(c!) num_padded, Tensor(d!) inv, Tensor(e!) tile_expert) -> ()");
  m.def(
      "moe_gemm(Tensor(a!) out, Tensor a, Tensor w, Tensor sorted_ids, Tensor tile_expert, "
      "int n_flat, int topk, bool gather) -> ()");
  m.def("moe_combine(Tensor y, Tensor wts, Tensor inv, Tensor(a!) out) -> ()");
  m.def(
      "moe_dgemm(Tensor(a!) out, Tensor a, Tensor w, Tensor sorted_ids, Tensor tile_expert, "
      "int n_flat, int topk, bool gather, bool silu, int pf, int bm=32, int splitk=1) -> ()");
  m.def(
      "moe_combine_split(Tensor partials, Tensor wts, Tensor inv, Tensor(a!) out, int splitk, "
      "int rows) -> ()");
  m.def("kv_gather(Tensor cache, Tensor block_ids, Tensor(a!) out) -> ()");
  m.def("kv_scatter(Tensor buf, Tensor(a!) cache, Tensor block_ids) -> ()");
  m.def("embedding(Tensor ids, Tensor table, Tensor(a!) out, int vocab_start, int vocab_end) -> ()");
  m.def("embedding_prep(Tensor ids, Tensor table, Tensor ln, Tensor(a!) residual, "
        "Tensor(b!) a_out, Tensor(c!) ss_out, Tensor(d!) zbuf, int vocab_start, "
        "int vocab_end) -> ()");
}

TORCH_LIBRARY_IMPL(akap, CompositeExplicitAutograd, m) {
  m.impl("gemm_splitk", &gemm_splitk);
  m.impl("dgemm_ok", &dgemm_ok);
  m.impl("car_create", &car_create);
  m.impl("car_ipc_handles", &car_ipc_handles);
  m.impl("car_open", &car_open);
  m.impl("car_error", &car_error);
  m.impl("car_error_word", &car_error_word);
  m.impl("car_link_local", &car_link_local);
  m.impl("car_destroy", &car_destroy);
  m.impl("ipc_open", &ipc_open);
  m.impl("ipc_close", &ipc_close);
  m.impl("h2d_stage", &h2d_stage);  // pinned CPU source + device destination
}

TORCH_LIBRARY_IMPL(akap, CUDA, m) {
  m.impl("rmsnorm", &rmsnorm);
  m.impl("fused_add_rmsnorm", &fused_add_rmsnorm);
  m.impl("qk_norm_rope_cache", &qk_norm_rope_cache);
  m.impl("reshape_and_cache", &reshape_and_cache);
  m.impl("silu_and_mul", &silu_and_mul);
  m.impl("paged_attention_prefill", &paged_attention_prefill);
  m.impl("paged_attention_prefill_qprep", &paged_attention_prefill_qprep);
  m.impl("paged_attention_decode", &paged_attention_decode);
  m.impl("paged_attention_decode_fused", &paged_attention_decode_fused);
  m.impl("sample", &sample);
  m.impl("apply_penalties", &apply_penalties);
  m.impl("argmax", &argmax);
  m.impl("gemm", &gemm);
  m.impl("dgemm", &dgemm);
  m.impl("wgemm", &wgemm);
  m.impl("pgemm", &pgemm);
  m.impl("kgemm", &kgemm);
  m.impl("moe_topk_softmax", &moe_topk_softmax);
  m.impl("moe_router_topk", &moe_router_topk);
  m.impl("moe_align", &moe_align);
  m.impl("moe_gemm", &moe_gemm);
  m.impl("moe_combine", &moe_combine);
  m.impl("moe_dgemm", &moe_dgemm);
  m.impl("moe_combine_split", &moe_combine_split);
  m.impl("car_all_reduce", &car_all_reduce);
  m.impl("l2_prefetch", &l2_prefetch);
  m.impl("car_all_reduce_multi", &car_all_reduce_multi);
  m.impl("car_all_reduce_resnorm", &car_all_reduce_resnorm);
  m.impl("kv_gather", &kv_gather);
  m.impl("kv_scatter", &kv_scatter);
  m.impl("kv_pull", &kv_pull);
  m.impl("car_all_gather", &car_all_gather);
  m.impl("car_broadcast", &car_broadcast);
  m.impl("car_all_to_all", &car_all_to_all);
  m.impl("ipc_export", &ipc_export);
  m.impl("embedding", &embedding);
  m.impl("embedding_prep", &embedding_prep);
}
