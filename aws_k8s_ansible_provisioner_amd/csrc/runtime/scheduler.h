// Continuous-batching scheduler core (host side, C++).
//
// Per engine step it picks the work, allocates KV blocks, and writes the flattened
// batch description (token ids, positions, paged-cache slots, block tables, cu-seqlens,
// attention tile map, logits rows) straight into caller-owned pinned buffers, so the
// Python engine loop does no per-token work.  Policy:
//   * mixed batching (default): every running decode gets its token in the same step as the
//     prefill chunks (the decode rows lead the flattened batch: [0, num_decode)), so a
//     running decode does not stall behind prefills.  Under a prefill BACKLOG (more pending
//     prompt tokens than `mix_backlog_steps` steps' budget -- a burst of arrivals) the step
//     stays prefill-first, which minimises TTFT while the queue drains, but never for more
//     than `max_decode_stall_steps` consecutive steps;
//   * mixed_batching = false: prefill-first (a step is pure prefill while any is pending);
//   * a step with no prefill work is a pure decode step (hipGraph replay);
//   * out of KV blocks -> preempt the youngest running sequence (recompute later);
//   * P/D prefill side: KV blocks held for a transfer expire after held_kv_ttl_s.
#pragma once

#include <cstdint>
#include <deque>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "block_manager.h"

namespace akap_rt {

enum ReqStatus : int { WAITING = 0, RUNNING = 1, FINISHED = 2, PENDING_KV = 3 };
enum FinishReason : int { NOT_FINISHED = 0, FINISH_LENGTH = 1, FINISH_STOP = 2, FINISH_ABORT = 3 };

struct Request {
  int64_t id = 0;
  std::vector<int32_t> tokens;  // prompt + generated
  int num_prompt = 0;
  int max_tokens = 16;
  int min_tokens = 0;
  bool ignore_eos = false;
  std::vector<int32_t> stop_ids;
  int num_computed = 0;  // tokens whose K/V are in the cache
  int num_cached = 0;    // prefix-cache hit tokens (first schedule)
  std::vector<int32_t> blocks;
  std::vector<uint64_t> hashes;  // hashes of full, published blocks
  int status = WAITING;
  int finish = NOT_FINISHED;
  int num_preempt = 0;
  bool prefix_checked = false;
  // sampling parameters (consumed by the on-GPU sampler, indexed per sample row)
  float temperature = 0.f;
  float top_p = 1.f;
  int top_k = 0;
  int64_t seed = 0;
  bool stream = false;  // report every token (else only first token + finish)
  bool hold_kv = false; // P/D prefill side: keep KV blocks after finishing (for transfer)
  // V-tail slot (the GPU keeps this sequence's partial 8-token V group there): -2 = not yet
  // assigned, -1 = none (pool empty / tails off); held from first schedule to finish/preempt
  int tail_slot = -2;
  int num_generated() const { return (int)tokens.size() - num_prompt; }
};

struct SchedConfig {
  int max_num_seqs = 256;
  int max_num_batched_tokens = 8192;
  int max_model_len = 4096;
  int block_size = 32;
  int gqa_group = 1;      // q heads per kv head (prefill tile map)
  int tile_rows = 64;     // flattened query rows per prefill attention workgroup
  // steps whose every prefill chunk has <= short_rows flattened q rows (chunk tokens x
  // gqa_group) use tile_rows_short instead (0: off).  The engine sets 256 / 128: with the
  // longest-first grid the 8-wave 256-row kernel wins on long chunks, the 128-row one on
  // short prompts with small GQA groups (profiles/r6_prefill_tile_order.md)
  int tile_rows_short = 0;
  int short_rows = 1024;
  int eos_id = -1;
  int max_blocks_per_seq = 128;
  bool mixed_batching = true;
  int mix_backlog_steps = 1;       // mix when pending prefill <= this many steps' budget
  int max_decode_stall_steps = 8;  // ... or after this many prefill-only steps in a row
  double held_kv_ttl_s = 120.0;  // P/D: held KV never pulled by a decode engine is freed
  int num_tail_slots = 0;        // V-tail slots (0: tails off, every row gets -1)
};

// Views into caller buffers (numpy, pinned).  Sizes are checked by the binding.
struct BatchBuffers {
  int64_t* input_ids;
  int64_t* positions;
  int64_t* slots;
  int32_t* seq_lens;
  int32_t* q_start;
  int32_t* block_tables;  // [max_num_seqs, max_blocks_per_seq]
  int32_t* tile_seq;
  int32_t* tile_row;
  int64_t* logits_idx;
  int64_t* req_ids;       // per scheduled seq
  int32_t* sample_mask;   // per scheduled seq: 1 if its last token is sampled
  // per sample row
  float* temperature;
  float* top_p;
  int32_t* top_k;
  int64_t* seeds;
  int32_t* steps;
  int32_t* tail_slot;     // per token: its sequence's V-tail slot (nullptr: not staged)
  int cap_tokens, cap_tiles;
};

struct StepInfo {
  int is_prefill = 0;
  int num_seqs = 0;
  int num_tokens = 0;
  int num_tiles = 0;
  int num_samples = 0;
  int max_seq_len = 0;
  int num_preempted = 0;
  int num_decode = 0;  // leading single-token decode rows (all rows of a pure decode step)
  int tile_rows = 0;   // prefill tile map granularity of this step
};

class Scheduler {
 public:
  Scheduler(const SchedConfig& cfg, int num_blocks, bool prefix_cache);

  void add_request(int64_t id, const std::vector<int32_t>& prompt, int max_tokens, int min_tokens,
                   bool ignore_eos, const std::vector<int32_t>& stop_ids, float temperature = 0.f,
                   float top_p = 1.f, int top_k = 0, int64_t seed = 0, bool stream = false);
  bool abort_request(int64_t id);
  StepInfo schedule(BatchBuffers& buf);
  // Decode lookahead (async scheduling): called while the pure decode step just scheduled
  // (or looked ahead) is still running on the GPU and BEFORE its update().  Builds the next
  // decode step assuming every row of the in-flight step appends its (not yet known) token:
  // input ids are not written -- src_rows[j] names the in-flight row whose sampled token is
  // row j's input, and the device gathers it.  Rows whose pending token finishes them by
  // length are left out; a row that turns out to finish by EOS/stop (or is aborted) computes
  // one discarded token (its KV lands in its own, already freed blocks before any reuse:
  // stream order).  Returns num_seqs = 0 when the next step must be a normal one (waiting
  // requests that a free sequence slot could admit, a running sequence outside the in-flight
  // batch, no KV blocks, nothing left).
  StepInfo schedule_lookahead(BatchBuffers& buf, int64_t* src_rows);
  // tokens[i] is the sample for the i-th sampled sequence of the last step.
  // Emits (id, token, finish_reason, is_first) events only for sequences that got their
  // first token, finished, or stream -- O(events) host work per step, not O(batch).
  void update(const int64_t* tokens, int n, std::vector<int64_t>& out_ids,
              std::vector<int32_t>& out_tokens, std::vector<int32_t>& out_finish,
              std::vector<int32_t>& out_first);

  // tokens the last update() appended to live sequences (rows of requests that finished or
  // were aborted while the step was in flight are computed but not counted)
  int last_appended() const { return last_appended_; }
  int num_waiting() const { return (int)waiting_.size(); }
  int num_running() const { return (int)running_.size(); }
  bool has_work() const {
    return !waiting_.empty() || !running_.empty() || !sched_finished_.empty() ||
           !pending_.empty();
  }
  const BlockManager& blocks() const { return bm_; }
  BlockManager& blocks_mut() { return bm_; }
  const Request* get(int64_t id) const;
  std::vector<int32_t> block_table(int64_t id) const;
  int64_t total_preemptions() const { return preemptions_; }
  const SchedConfig& config() const { return cfg_; }
  // drop a finished request's bookkeeping (called by the engine after delivery)
  void release(int64_t id);

  // ---- disaggregated prefill/decode ----
  void set_hold_kv(int64_t id, bool hold);
  // prefill side: blocks of a finished hold_kv request (kept until free_held)
  std::vector<int32_t> held_blocks(int64_t id) const;
  void free_held(int64_t id);
  // a send of this held KV starts: the entry leaves the TTL-tracked held set (expire_held and
  // free_held -- a /kv/release from a decode side that gave up -- no longer touch it) and its
  // blocks stay owned until finish_transfer(), which the send's completion calls.  Returns the
  // blocks (empty: nothing held under this id, e.g. already expired)
  std::vector<int32_t> take_held(int64_t id);
  void finish_transfer(int64_t id);
  size_t num_in_transfer() const { return in_transfer_.size(); }
  // decode side: register a request whose prompt KV arrives from a prefill engine.
  // tokens = prompt + first generated token.  Allocates the prompt's blocks and
  // returns them (empty if the pool is short); the request is not scheduled until
  // activate().
  std::vector<int32_t> reserve_prefilled(int64_t id, const std::vector<int32_t>& tokens,
                                         int num_prompt, int max_tokens, int min_tokens,
                                         bool ignore_eos, const std::vector<int32_t>& stop_ids,
                                         float temperature, float top_p, int top_k,
                                         int64_t seed, bool stream);
  void activate(int64_t id);
  // P/D streamed hand-off: blocks are reserved (and filled chunk by chunk) before the prefill
  // has sampled the first token; it is set here, before activate()
  void set_first_token(int64_t id, int32_t tok);
  // V-tail slot of a request (assigning one if it has none yet; -1 = no tail)
  int tail_slot(int64_t id);
  int num_free_tail_slots() const { return (int)free_tails_.size(); }
  size_t num_held() const { return held_.size(); }
  // free every held-KV entry whose deadline passed (schedule() calls it with the steady
  // clock); returns the number expired
  int expire_held(double now_s);
  int64_t held_expired_total() const { return held_expired_; }
  static double now_s();

 private:
  bool ensure_blocks(Request& r, int num_tokens);
  void schedule_decodes(std::vector<std::pair<Request*, int>>& sched, StepInfo& info,
                        int& budget);
  void schedule_prefills(std::vector<std::pair<Request*, int>>& sched, int& budget);
  void publish_full_blocks(Request& r);
  void preempt(Request& r);
  void finish(Request& r, int reason);
  int32_t tail_of(Request& r);
  void drop_tail(Request& r);

  SchedConfig cfg_;
  BlockManager bm_;
  std::unordered_map<int64_t, std::unique_ptr<Request>> reqs_;
  std::deque<Request*> waiting_;
  std::vector<Request*> running_;
  // ids of the sampled rows of every scheduled step whose update() is still due, oldest
  // first (one entry normally; two while a lookahead step is in flight).  Ids, not pointers:
  // a request may finish, be aborted or released while a step that holds it is in flight.
  std::deque<std::vector<int64_t>> pending_;
  bool last_pure_decode_ = false;  // the newest pending step is a pure decode step
  // requests the scheduler itself had to finish (KV pool can never hold them); reported by
  // the next update() as events with token -1
  std::vector<std::pair<int64_t, int>> sched_finished_;
  struct HeldKV {
    std::vector<int32_t> blocks;
    double deadline;
  };
  std::unordered_map<int64_t, HeldKV> held_;
  std::unordered_map<int64_t, std::vector<int32_t>> in_transfer_;  // held KV being sent
  std::vector<int32_t> free_tails_;  // V-tail slot pool (LIFO)
  int64_t preemptions_ = 0;
  int64_t held_expired_ = 0;
  int prefill_only_run_ = 0;  // consecutive prefill-only steps while decodes were waiting
  int last_appended_ = 0;     // tokens appended to live sequences by the last update()
};

}  // namespace akap_rt
