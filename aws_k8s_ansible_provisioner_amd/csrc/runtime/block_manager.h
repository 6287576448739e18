// Paged KV-cache block manager (host side, C++).
//
// Sized for MI355X: the engine gives the cache most of the 288 GB HBM, i.e. hundreds
// of thousands of blocks, so every operation here is O(blocks touched), never O(pool).
//  * free pool: LIFO stack (recently freed blocks are warm in the Infinity Cache)
//  * prefix cache: full blocks are content-addressed by a chained 64-bit hash of their
//    tokens; a freed cached block parks in an LRU "evictable" list and is revived on a
//    hit, or recycled when the free stack runs dry.
#pragma once

#include <cstdint>
#include <list>
#include <unordered_map>
#include <vector>

namespace akap_rt {

class BlockManager {
 public:
  BlockManager(int num_blocks, int block_size, bool enable_prefix_cache);

  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  int num_free() const { return (int)free_.size() + (int)lru_.size(); }
  double usage() const { return 1.0 - (double)num_free() / (double)num_blocks_; }

  // Chained hash of one full block.
  static uint64_t hash_block(uint64_t parent, const int32_t* toks, int n);

  // Longest run of cached full blocks for `tokens`; returns hit blocks (ref-counted)
  // and their hashes.  Does not allocate anything new.
  int match_prefix(const std::vector<int32_t>& tokens, int max_tokens, std::vector<int32_t>& blocks,
                   std::vector<uint64_t>& hashes);
  // Take one fresh block (ref=1). -1 if none.
  int allocate();
  // Release a sequence's blocks (reverse order so tails are evicted first).
  void free_blocks(const std::vector<int32_t>& blocks);
  // Publish a now-full block under `h` (prefix caching).
  void register_full(int block, uint64_t h);
  void reset_prefix_cache();

  int64_t prefix_hits() const { return hits_; }
  int64_t prefix_queries() const { return queries_; }

 private:
  void touch_evictable(int b);
  int num_blocks_, block_size_;
  bool prefix_;
  std::vector<int32_t> free_;
  std::vector<int32_t> ref_;
  std::vector<uint64_t> hash_of_;  // 0 = not cached
  std::vector<uint8_t> in_lru_;
  std::list<int32_t> lru_;
  std::vector<std::list<int32_t>::iterator> lru_pos_;
  std::unordered_map<uint64_t, int32_t> cached_;
  int64_t hits_ = 0, queries_ = 0;
};

}  // namespace akap_rt
