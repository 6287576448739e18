#include "scheduler.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <stdexcept>

namespace akap_rt {

namespace {
// Orders the step's prefill tile map by ascending causal work: a tile's cost is the key count
// its last q row attends to (the chunk's context plus its furthest token).  The prefill
// attention kernel walks one flat (tile, kv head) grid back to front, so this makes the
// launch longest-first over the whole grid and leaves only the shortest tiles for its tail
// (attention.hip, paged_attn_prefill_fa_kernel).  Stable: equal-work tiles keep map order.
void sort_tiles_by_work(BatchBuffers& buf, int tiles, int step_rows, int G) {
  static const bool on = [] {  // AKAP_TILE_SORT=0: keep map order (A/B knob)
    const char* e = std::getenv("AKAP_TILE_SORT");
    return e == nullptr || std::atoi(e) != 0;
  }();
  if (tiles < 2 || !on) return;
  std::vector<std::pair<int, int>> key(tiles);  // (work, original index)
  for (int i = 0; i < tiles; ++i) {
    const int s = buf.tile_seq[i];
    const int q = buf.q_start[s + 1] - buf.q_start[s];
    const int last_tok = std::min(q, (buf.tile_row[i] + step_rows + G - 1) / G);
    key[i] = {buf.seq_lens[s] - q + last_tok, i};
  }
  std::stable_sort(key.begin(), key.end(),
                   [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<int32_t> ts(tiles), tr(tiles);
  for (int i = 0; i < tiles; ++i) {
    ts[i] = buf.tile_seq[key[i].second];
    tr[i] = buf.tile_row[key[i].second];
  }
  std::copy(ts.begin(), ts.end(), buf.tile_seq);
  std::copy(tr.begin(), tr.end(), buf.tile_row);
}
}  // namespace

Scheduler::Scheduler(const SchedConfig& cfg, int num_blocks, bool prefix_cache)
    : cfg_(cfg), bm_(num_blocks, cfg.block_size, prefix_cache) {
  if (cfg_.max_blocks_per_seq * cfg_.block_size < cfg_.max_model_len)
    throw std::invalid_argument("max_blocks_per_seq * block_size < max_model_len");
  for (int i = cfg_.num_tail_slots - 1; i >= 0; --i) free_tails_.push_back(i);
}

int32_t Scheduler::tail_of(Request& r) {
  if (r.tail_slot == -2) {
    if (free_tails_.empty()) {
      r.tail_slot = -1;  // no slot: this sequence keeps the plain V cache write path
    } else {
      r.tail_slot = free_tails_.back();
      free_tails_.pop_back();
    }
  }
  return r.tail_slot;
}

void Scheduler::drop_tail(Request& r) {
  // a step still in flight may write the old slot: it runs before any step that hands the
  // slot to another sequence (one stream), so the slot is free for reuse at once
  if (r.tail_slot >= 0) free_tails_.push_back(r.tail_slot);
  r.tail_slot = -2;
}

int Scheduler::tail_slot(int64_t id) {
  auto it = reqs_.find(id);
  return it == reqs_.end() ? -1 : tail_of(*it->second);
}

void Scheduler::add_request(int64_t id, const std::vector<int32_t>& prompt, int max_tokens,
                            int min_tokens, bool ignore_eos, const std::vector<int32_t>& stop_ids,
                            float temperature, float top_p, int top_k, int64_t seed,
                            bool stream) {
  if (reqs_.count(id)) throw std::invalid_argument("duplicate request id");
  if (prompt.empty()) throw std::invalid_argument("empty prompt");
  if ((int)prompt.size() >= cfg_.max_model_len)
    throw std::invalid_argument("prompt longer than max_model_len");
  auto r = std::make_unique<Request>();
  r->id = id;
  r->tokens = prompt;
  r->num_prompt = (int)prompt.size();
  r->max_tokens = std::max(1, max_tokens);
  r->min_tokens = min_tokens;
  r->ignore_eos = ignore_eos;
  r->stop_ids = stop_ids;
  r->temperature = temperature;
  r->top_p = top_p;
  r->top_k = top_k;
  r->seed = seed;
  r->stream = stream;
  waiting_.push_back(r.get());
  reqs_.emplace(id, std::move(r));
}

const Request* Scheduler::get(int64_t id) const {
  auto it = reqs_.find(id);
  return it == reqs_.end() ? nullptr : it->second.get();
}

std::vector<int32_t> Scheduler::block_table(int64_t id) const {
  auto r = get(id);
  return r ? r->blocks : std::vector<int32_t>{};
}

void Scheduler::release(int64_t id) {
  auto it = reqs_.find(id);
  if (it != reqs_.end() && it->second->status == FINISHED) reqs_.erase(it);
}

void Scheduler::set_hold_kv(int64_t id, bool hold) {
  auto it = reqs_.find(id);
  if (it != reqs_.end()) it->second->hold_kv = hold;
}

std::vector<int32_t> Scheduler::held_blocks(int64_t id) const {
  auto it = held_.find(id);
  return it == held_.end() ? std::vector<int32_t>{} : it->second.blocks;
}

void Scheduler::free_held(int64_t id) {
  auto it = held_.find(id);
  if (it == held_.end()) return;
  bm_.free_blocks(it->second.blocks);
  held_.erase(it);
}

std::vector<int32_t> Scheduler::take_held(int64_t id) {
  auto it = held_.find(id);
  if (it == held_.end()) return {};
  std::vector<int32_t> b = std::move(it->second.blocks);
  held_.erase(it);
  auto& slot = in_transfer_[id];
  if (!slot.empty()) bm_.free_blocks(slot);  // defensive: an id is never sent twice
  slot = b;
  return b;
}

void Scheduler::finish_transfer(int64_t id) {
  auto it = in_transfer_.find(id);
  if (it == in_transfer_.end()) return;
  bm_.free_blocks(it->second);
  in_transfer_.erase(it);
}

double Scheduler::now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int Scheduler::expire_held(double now) {
  int n = 0;
  for (auto it = held_.begin(); it != held_.end();) {
    if (it->second.deadline <= now) {
      bm_.free_blocks(it->second.blocks);
      it = held_.erase(it);
      ++n;
    } else {
      ++it;
    }
  }
  held_expired_ += n;
  return n;
}

std::vector<int32_t> Scheduler::reserve_prefilled(
    int64_t id, const std::vector<int32_t>& tokens, int num_prompt, int max_tokens,
    int min_tokens, bool ignore_eos, const std::vector<int32_t>& stop_ids, float temperature,
    float top_p, int top_k, int64_t seed, bool stream) {
  if (reqs_.count(id)) throw std::invalid_argument("duplicate request id");
  if (num_prompt <= 0 || (int)tokens.size() != num_prompt + 1)
    throw std::invalid_argument("reserve_prefilled: tokens must be prompt + first token");
  if ((int)tokens.size() >= cfg_.max_model_len)
    throw std::invalid_argument("prompt longer than max_model_len");
  auto r = std::make_unique<Request>();
  r->id = id;
  r->tokens = tokens;
  r->num_prompt = num_prompt;
  r->max_tokens = std::max(1, max_tokens);
  r->min_tokens = min_tokens;
  r->ignore_eos = ignore_eos;
  r->stop_ids = stop_ids;
  r->temperature = temperature;
  r->top_p = top_p;
  r->top_k = top_k;
  r->seed = seed;
  r->stream = stream;
  r->prefix_checked = true;
  if (!ensure_blocks(*r, num_prompt)) {
    if (!r->blocks.empty()) bm_.free_blocks(r->blocks);
    return {};
  }
  r->num_computed = num_prompt;
  r->status = PENDING_KV;
  std::vector<int32_t> out = r->blocks;
  reqs_.emplace(id, std::move(r));
  return out;
}

void Scheduler::set_first_token(int64_t id, int32_t tok) {
  auto it = reqs_.find(id);
  if (it == reqs_.end() || it->second->status != PENDING_KV) return;
  it->second->tokens.back() = tok;
}

void Scheduler::activate(int64_t id) {
  auto it = reqs_.find(id);
  if (it == reqs_.end() || it->second->status != PENDING_KV) return;
  it->second->status = RUNNING;
  running_.push_back(it->second.get());
  tail_of(*it->second);  // the engine fills the tail from the received KV right after
}

bool Scheduler::abort_request(int64_t id) {
  auto it = reqs_.find(id);
  if (it == reqs_.end()) return false;
  Request* r = it->second.get();
  if (r->status == FINISHED) return false;
  if (r->status == WAITING) {
    waiting_.erase(std::remove(waiting_.begin(), waiting_.end(), r), waiting_.end());
  } else if (r->status == PENDING_KV) {
  } else {
    running_.erase(std::remove(running_.begin(), running_.end(), r), running_.end());
  }
  finish(*r, FINISH_ABORT);  // its rows in pending steps are skipped by update()
  return true;
}

void Scheduler::finish(Request& r, int reason) {
  if (r.hold_kv && reason != FINISH_ABORT && !r.blocks.empty()) {
    // P/D: ownership moves to the transfer agent until a decode engine pulls the KV
    // (/kv/push -> free_held), releases it (/kv/release), or the TTL runs out
    held_[r.id] = HeldKV{r.blocks, now_s() + cfg_.held_kv_ttl_s};
  } else if (!r.blocks.empty()) {
    bm_.free_blocks(r.blocks);
  }
  r.blocks.clear();
  r.hashes.clear();
  drop_tail(r);
  r.status = FINISHED;
  r.finish = reason;
}

bool Scheduler::ensure_blocks(Request& r, int num_tokens) {
  const int need = (num_tokens + cfg_.block_size - 1) / cfg_.block_size;
  if (need > cfg_.max_blocks_per_seq) return false;
  while ((int)r.blocks.size() < need) {
    const int b = bm_.allocate();
    if (b < 0) return false;
    r.blocks.push_back(b);
  }
  return true;
}

void Scheduler::publish_full_blocks(Request& r) {
  const int bs = cfg_.block_size;
  // a lookahead step counts the in-flight token as computed before it is in r.tokens
  const int done = std::min(r.num_computed, (int)r.tokens.size());
  while ((int)r.hashes.size() < (int)r.blocks.size() && ((int)r.hashes.size() + 1) * bs <= done) {
    const int i = (int)r.hashes.size();
    const uint64_t parent = i ? r.hashes[i - 1] : 0;
    const uint64_t h = BlockManager::hash_block(parent, r.tokens.data() + i * bs, bs);
    bm_.register_full(r.blocks[i], h);
    r.hashes.push_back(h);
  }
}

void Scheduler::preempt(Request& r) {
  bm_.free_blocks(r.blocks);
  drop_tail(r);  // recomputed from scratch: the prefill rewrites the tail of a new slot
  r.blocks.clear();
  r.hashes.clear();
  r.num_computed = 0;
  r.prefix_checked = false;
  r.status = WAITING;
  r.num_preempt += 1;
  ++preemptions_;
  running_.erase(std::remove(running_.begin(), running_.end(), &r), running_.end());
  waiting_.push_front(&r);
}

void Scheduler::schedule_prefills(std::vector<std::pair<Request*, int>>& sched, int& budget) {
  // running sequences with more than one uncomputed token: the next chunk of their prompt
  for (Request* r : running_) {
    const int remaining = (int)r->tokens.size() - r->num_computed;
    if (remaining <= 1 || budget <= 0) continue;
    if ((int)sched.size() >= cfg_.max_num_seqs) break;
    const int q = std::min(remaining, budget);
    if (!ensure_blocks(*r, r->num_computed + q)) break;
    sched.emplace_back(r, q);
    budget -= q;
  }
  // admit waiting requests (FCFS) while budget, sequence slots and KV blocks last
  while (!waiting_.empty() && budget > 0 &&
         (int)running_.size() < cfg_.max_num_seqs && (int)sched.size() < cfg_.max_num_seqs) {
    Request* r = waiting_.front();
    if (!r->prefix_checked) {
      r->prefix_checked = true;
      std::vector<int32_t> hb;
      std::vector<uint64_t> hh;
      const int hit = bm_.match_prefix(r->tokens, (int)r->tokens.size() - 1, hb, hh);
      r->blocks = hb;
      r->hashes = hh;
      r->num_computed = hit;
      r->num_cached = hit;
    }
    const int remaining = (int)r->tokens.size() - r->num_computed;
    const int q = std::min(remaining, budget);
    if (!ensure_blocks(*r, r->num_computed + q)) {
      if (running_.empty() && sched.empty()) {
        // nothing holds blocks and it still does not fit: it never will
        waiting_.pop_front();
        finish(*r, FINISH_ABORT);
        sched_finished_.emplace_back(r->id, FINISH_ABORT);
        continue;
      }
      break;
    }
    waiting_.pop_front();
    r->status = RUNNING;
    running_.push_back(r);
    sched.emplace_back(r, q);
    budget -= q;
  }
}

void Scheduler::schedule_decodes(std::vector<std::pair<Request*, int>>& sched, StepInfo& info,
                                 int& budget) {
  // one token for every running sequence whose prompt is fully computed; oldest first,
  // preempt from the young end when the pool runs dry
  const int mb = cfg_.max_blocks_per_seq;
  size_t i = 0;
  while (i < running_.size()) {
    Request* r = running_[i];
    if ((int)sched.size() >= cfg_.max_num_seqs || budget <= 0) break;
    if ((int)r->tokens.size() - r->num_computed != 1) {  // still prefilling
      ++i;
      continue;
    }
    if (ensure_blocks(*r, r->num_computed + 1)) {
      sched.emplace_back(r, 1);
      --budget;
      ++i;
      continue;
    }
    // out of blocks (or seq too long): preempt the youngest other sequence
    Request* victim = running_.back();
    if ((int)r->blocks.size() >= mb || (victim == r && i == 0)) {
      // too long, or alone and the whole pool still cannot hold its next token:
      // end it here (length-capped) instead of preempting it forever
      finish(*r, FINISH_LENGTH);
      sched_finished_.emplace_back(r->id, FINISH_LENGTH);
      running_.erase(running_.begin() + i);
      continue;
    }
    // a victim already scheduled in this step is not preempted (its rows are written)
    bool scheduled = false;
    for (auto& e : sched) scheduled |= e.first == victim;
    if (scheduled) break;
    preempt(*victim);
    ++info.num_preempted;
    if (victim == r) break;
  }
}

StepInfo Scheduler::schedule(BatchBuffers& buf) {
  StepInfo info;
  pending_.clear();  // a normal step is only scheduled with nothing in flight
  std::vector<int64_t> sampled;
  if (!held_.empty()) expire_held(now_s());
  const int bs = cfg_.block_size;
  const int mb = cfg_.max_blocks_per_seq;
  std::vector<std::pair<Request*, int>> sched;  // (request, q_len)
  // prefill chunks get the whole token budget; the decode rows of a mixed step ride along
  // on top of it (one token each, at most max_num_seqs), so mixing never shrinks the
  // prefill chunks (TTFT) -- the token buffers hold budget + max_num_seqs rows
  int budget = std::min(cfg_.max_num_batched_tokens, buf.cap_tokens);

  // pending prompt tokens (waiting requests not yet prefix-matched count in full) and
  // whether any running sequence is in its decode phase
  int64_t backlog = 0;
  bool any_decode = false;
  for (Request* r : waiting_) backlog += (int)r->tokens.size() - r->num_computed;
  for (Request* r : running_) {
    const int rem = (int)r->tokens.size() - r->num_computed;
    if (rem > 1) backlog += rem;
    else any_decode = true;
  }
  const bool pending_prefill = backlog > 0;
  bool mix = pending_prefill && cfg_.mixed_batching && any_decode;
  if (mix && backlog > (int64_t)budget * cfg_.mix_backlog_steps &&
      prefill_only_run_ < cfg_.max_decode_stall_steps)
    mix = false;  // burst: drain the prefill queue first (TTFT), decodes wait a bounded time
  if (mix) {
    // mixed step: decodes first (they never stall behind a prefill), then prefill chunks
    int dbudget = std::max(0, std::min(cfg_.max_num_seqs, buf.cap_tokens - budget));
    schedule_decodes(sched, info, dbudget);
    info.num_decode = (int)sched.size();
    schedule_prefills(sched, budget);
  } else if (pending_prefill) {
    schedule_prefills(sched, budget);  // prefill-first policy
  }
  if (sched.empty()) {
    budget = std::min(cfg_.max_num_batched_tokens, buf.cap_tokens);
    schedule_decodes(sched, info, budget);
    info.num_decode = (int)sched.size();
  }
  info.is_prefill = (int)sched.size() > info.num_decode ? 1 : 0;
  // bounded decode stall: count steps that actually ran prefill rows while decodes waited
  // (a prefill-first step that fit no chunk fell back to pure decode: not a stall)
  prefill_only_run_ = (info.is_prefill && info.num_decode == 0 && any_decode)
                          ? prefill_only_run_ + 1 : 0;

  // ---------------- flatten ----------------
  int step_rows = cfg_.tile_rows;
  if (cfg_.tile_rows_short > 0 && info.is_prefill) {
    int longest = 0;
    for (size_t s = (size_t)info.num_decode; s < sched.size(); ++s)
      longest = std::max(longest, sched[s].second * cfg_.gqa_group);
    if (longest <= cfg_.short_rows) step_rows = cfg_.tile_rows_short;
  }
  info.tile_rows = step_rows;
  int T = 0, tiles = 0, ns = 0;
  for (size_t s = 0; s < sched.size(); ++s) {
    Request* r = sched[s].first;
    const int q = sched[s].second;
    if (T + q > buf.cap_tokens) throw std::runtime_error("token buffer too small");
    buf.q_start[s] = T;
    const int start = r->num_computed;
    for (int j = 0; j < q; ++j) {
      const int pos = start + j;
      buf.input_ids[T + j] = r->tokens[pos];
      buf.positions[T + j] = pos;
      buf.slots[T + j] = (int64_t)r->blocks[pos / bs] * bs + pos % bs;
    }
    if (buf.tail_slot != nullptr) {
      const int32_t ts = tail_of(*r);
      for (int j = 0; j < q; ++j) buf.tail_slot[T + j] = ts;
    }
    const int kv = start + q;
    buf.seq_lens[s] = kv;
    info.max_seq_len = std::max(info.max_seq_len, kv);
    int32_t* row = buf.block_tables + (size_t)s * mb;
    const int nb = (int)r->blocks.size();
    for (int b = 0; b < mb; ++b) row[b] = b < nb ? r->blocks[b] : 0;
    buf.req_ids[s] = r->id;
    if (info.is_prefill && (int)s >= info.num_decode) {  // decode rows: decode kernel
      const int rows = q * cfg_.gqa_group;
      for (int t0 = 0; t0 < rows; t0 += step_rows) {
        if (tiles >= buf.cap_tiles) throw std::runtime_error("tile buffer too small");
        buf.tile_seq[tiles] = (int)s;
        buf.tile_row[tiles] = t0;
        ++tiles;
      }
    }
    r->num_computed = kv;
    const bool sample = kv == (int)r->tokens.size();
    buf.sample_mask[s] = sample ? 1 : 0;
    if (sample) {
      buf.temperature[ns] = r->temperature;
      buf.top_p[ns] = r->top_p;
      buf.top_k[ns] = r->top_k;
      buf.seeds[ns] = r->seed;
      buf.steps[ns] = r->num_generated();
      buf.logits_idx[ns++] = T + q - 1;
      sampled.push_back(r->id);
    }
    T += q;
  }
  buf.q_start[sched.size()] = T;
  sort_tiles_by_work(buf, tiles, step_rows, cfg_.gqa_group);
  info.num_seqs = (int)sched.size();
  info.num_tokens = T;
  info.num_tiles = tiles;
  info.num_samples = ns;
  pending_.push_back(std::move(sampled));
  last_pure_decode_ = !info.is_prefill && info.num_seqs > 0;
  return info;
}

StepInfo Scheduler::schedule_lookahead(BatchBuffers& buf, int64_t* src_rows) {
  StepInfo info;
  if (pending_.size() != 1 || !last_pure_decode_ || !sched_finished_.empty()) return info;
  // waiting requests: only while every sequence slot is taken (a normal step could not admit
  // them either); a length finish in the in-flight step frees a slot -> normal step
  const bool queued = !waiting_.empty();
  if (queued && (int)running_.size() < cfg_.max_num_seqs) return info;
  const std::vector<int64_t>& prev = pending_.back();
  const int bs = cfg_.block_size;
  const int mb = cfg_.max_blocks_per_seq;
  std::vector<std::pair<Request*, int>> rows;  // (request, in-flight row)
  int live = 0;
  for (int i = 0; i < (int)prev.size(); ++i) {
    auto it = reqs_.find(prev[i]);
    if (it == reqs_.end() || it->second->status != RUNNING) continue;
    Request* r = it->second.get();
    ++live;
    // the in-flight step appends one token: does that token end r by length?
    const int gen_after = r->num_generated() + 1;
    const int len_after = (int)r->tokens.size() + 1;
    if (gen_after >= r->max_tokens || len_after >= cfg_.max_model_len) continue;
    rows.emplace_back(r, i);
  }
  // every running sequence must be in the in-flight batch (an activated P/D request or a
  // still-prefilling one needs a normal step)
  if (live != (int)running_.size() || rows.empty() || (int)rows.size() > cfg_.max_num_seqs)
    return info;
  if (queued && (int)rows.size() != live) return info;
  for (auto& e : rows)
    if (!ensure_blocks(*e.first, e.first->num_computed + 1)) return info;
  int ns = 0;
  for (auto& e : rows) {
    Request* r = e.first;
    const int pos = r->num_computed;  // position of the in-flight step's token
    buf.q_start[ns] = ns;
    buf.input_ids[ns] = -1;  // gathered on the device from the in-flight step's samples
    src_rows[ns] = e.second;
    buf.positions[ns] = pos;
    buf.slots[ns] = (int64_t)r->blocks[pos / bs] * bs + pos % bs;
    buf.seq_lens[ns] = pos + 1;
    if (buf.tail_slot != nullptr) buf.tail_slot[ns] = tail_of(*r);
    info.max_seq_len = std::max(info.max_seq_len, pos + 1);
    int32_t* row = buf.block_tables + (size_t)ns * mb;
    const int nb = (int)r->blocks.size();
    for (int b = 0; b < mb; ++b) row[b] = b < nb ? r->blocks[b] : 0;
    buf.req_ids[ns] = r->id;
    buf.sample_mask[ns] = 1;
    buf.temperature[ns] = r->temperature;
    buf.top_p[ns] = r->top_p;
    buf.top_k[ns] = r->top_k;
    buf.seeds[ns] = r->seed;
    buf.steps[ns] = r->num_generated() + 1;
    buf.logits_idx[ns] = ns;
    r->num_computed = pos + 1;
    ++ns;
  }
  buf.q_start[ns] = ns;
  std::vector<int64_t> sampled;
  sampled.reserve(ns);
  for (auto& e : rows) sampled.push_back(e.first->id);
  pending_.push_back(std::move(sampled));
  info.num_seqs = info.num_tokens = info.num_samples = info.num_decode = ns;
  return info;
}

void Scheduler::update(const int64_t* tokens, int n, std::vector<int64_t>& out_ids,
                       std::vector<int32_t>& out_tokens, std::vector<int32_t>& out_finish,
                       std::vector<int32_t>& out_first) {
  if (pending_.empty()) {
    if (n) throw std::invalid_argument("update() without a scheduled step");
  } else if (n != (int)pending_.front().size()) {
    throw std::invalid_argument("sample count mismatch");
  }
  std::vector<int64_t> sampled;
  if (!pending_.empty()) {
    sampled = std::move(pending_.front());
    pending_.pop_front();
  }
  for (const auto& f : sched_finished_) {
    out_ids.push_back(f.first);
    out_tokens.push_back(-1);
    out_finish.push_back(f.second);
    out_first.push_back(0);
  }
  sched_finished_.clear();
  last_appended_ = 0;
  for (Request* r : running_) publish_full_blocks(*r);
  for (int i = 0; i < n; ++i) {
    auto it = reqs_.find(sampled[i]);
    // finished (EOS/stop in an earlier update, aborted) or released while this step was in
    // flight: its row was computed and is discarded
    if (it == reqs_.end() || it->second->status != RUNNING) continue;
    Request* r = it->second.get();
    const int32_t tok = (int32_t)tokens[i];
    r->tokens.push_back(tok);
    ++last_appended_;
    int reason = NOT_FINISHED;
    const int gen = r->num_generated();
    if (!r->ignore_eos && gen > r->min_tokens - 1 && tok == cfg_.eos_id) reason = FINISH_STOP;
    if (reason == NOT_FINISHED && gen >= r->min_tokens)
      for (int32_t s : r->stop_ids)
        if (s == tok) { reason = FINISH_STOP; break; }
    if (reason == NOT_FINISHED &&
        (gen >= r->max_tokens || (int)r->tokens.size() >= cfg_.max_model_len))
      reason = FINISH_LENGTH;
    const bool first = gen == 1;
    if (first || reason != NOT_FINISHED || r->stream) {
      out_ids.push_back(r->id);
      out_tokens.push_back(tok);
      out_finish.push_back(reason);
      out_first.push_back(first ? 1 : 0);
    }
    if (reason != NOT_FINISHED) {
      running_.erase(std::remove(running_.begin(), running_.end(), r), running_.end());
      finish(*r, reason);
    }
  }
}

}  // namespace akap_rt
