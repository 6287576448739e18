#include "block_manager.h"

#include <stdexcept>

namespace akap_rt {

BlockManager::BlockManager(int num_blocks, int block_size, bool enable_prefix_cache)
    : num_blocks_(num_blocks), block_size_(block_size), prefix_(enable_prefix_cache) {
  if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("bad block pool");
  free_.reserve(num_blocks);
  // block 0 is handed out last so padded block-table entries (0) stay harmless
  for (int b = num_blocks - 1; b >= 0; --b) free_.push_back(b);
  ref_.assign(num_blocks, 0);
  hash_of_.assign(num_blocks, 0);
  in_lru_.assign(num_blocks, 0);
  lru_pos_.resize(num_blocks);
}

uint64_t BlockManager::hash_block(uint64_t parent, const int32_t* toks, int n) {
  // FNV-1a over (parent, tokens) followed by a splitmix finaliser; never returns 0.
  uint64_t h = 1469598103934665603ull ^ parent;
  for (int i = 0; i < n; ++i) {
    h ^= (uint32_t)toks[i];
    h *= 1099511628211ull;
  }
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h ? h : 1;
}

int BlockManager::match_prefix(const std::vector<int32_t>& tokens, int max_tokens,
                               std::vector<int32_t>& blocks, std::vector<uint64_t>& hashes) {
  if (!prefix_) return 0;
  queries_ += max_tokens;  // token counts, like vllm:prefix_cache_{queries,hits}_total
  uint64_t parent = 0;
  int matched = 0;
  const int nfull = max_tokens / block_size_;
  for (int i = 0; i < nfull; ++i) {
    const uint64_t h = hash_block(parent, tokens.data() + i * block_size_, block_size_);
    auto it = cached_.find(h);
    if (it == cached_.end()) break;
    const int b = it->second;
    if (in_lru_[b]) {
      lru_.erase(lru_pos_[b]);
      in_lru_[b] = 0;
    }
    ref_[b] += 1;
    blocks.push_back(b);
    hashes.push_back(h);
    parent = h;
    matched += block_size_;
  }
  hits_ += matched;
  return matched;
}

int BlockManager::allocate() {
  int b;
  if (!free_.empty()) {
    b = free_.back();
    free_.pop_back();
  } else if (!lru_.empty()) {
    b = lru_.front();
    lru_.pop_front();
    in_lru_[b] = 0;
    auto it = cached_.find(hash_of_[b]);
    if (it != cached_.end() && it->second == b) cached_.erase(it);
    hash_of_[b] = 0;
  } else {
    return -1;
  }
  ref_[b] = 1;
  return b;
}

void BlockManager::touch_evictable(int b) {
  lru_.push_back(b);
  lru_pos_[b] = std::prev(lru_.end());
  in_lru_[b] = 1;
}

void BlockManager::free_blocks(const std::vector<int32_t>& blocks) {
  for (auto it = blocks.rbegin(); it != blocks.rend(); ++it) {
    const int b = *it;
    if (b < 0 || b >= num_blocks_ || ref_[b] <= 0) throw std::logic_error("double free of KV block");
    if (--ref_[b] == 0) {
      if (prefix_ && hash_of_[b] != 0)
        touch_evictable(b);
      else
        free_.push_back(b);
    }
  }
}

void BlockManager::register_full(int block, uint64_t h) {
  if (!prefix_ || hash_of_[block] != 0) return;
  auto it = cached_.find(h);
  if (it != cached_.end()) return;  // an identical block is already published
  cached_.emplace(h, block);
  hash_of_[block] = h;
}

void BlockManager::reset_prefix_cache() {
  for (int b : lru_) {
    in_lru_[b] = 0;
    hash_of_[b] = 0;
    free_.push_back(b);
  }
  lru_.clear();
  cached_.clear();
  for (auto& h : hash_of_) h = 0;
}

}  // namespace akap_rt
