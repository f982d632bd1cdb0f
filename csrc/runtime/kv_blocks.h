// Paged KV-cache block allocator + block-granular radix prefix cache.
//
// Realises the reference's spec'd KV Cache Manager (Req 4, requirements.md:63-74;
// design.md:363-413; Properties 9-12) on HBM pages instead of an in-RAM LRU map:
//   * prefix reuse (design.md:395 get_prefix): match() walks the radix tree one
//     full page (block_size tokens) at a time and returns the shared page ids.
//   * LRU eviction (Req 4.2 / Property 10): only pages referenced by nothing but
//     the cache are evictable; leaves are evicted oldest-`last_access` first,
//     parents become leaves as children go. The cache is also held under
//     `max_cached_blocks` (= memory_threshold * pool, design.md:371 default 0.8).
//   * access timestamps (Req 4.3 / Property 11): every node on a hit path gets
//     last_access = tick (monotone).
//   * counters (design.md:405-412): hits/misses (in tokens and lookups),
//     evictions, entries.
// Pages are immutable once they enter the cache (only FULL pages are inserted;
// a sequence only appends into its own tail page).
#pragma once

#include <cstdint>
#include <memory>
#include <set>
#include <unordered_map>
#include <utility>
#include <vector>

namespace xgs {

class BlockAllocator {
 public:
  explicit BlockAllocator(int num_blocks);
  int alloc();  // -1 when exhausted; returned page has refcount 1
  void incref(int b);
  void decref(int b);  // refcount 0 -> back on the free list
  int refcount(int b) const { return ref_[b]; }
  int num_free() const { return static_cast<int>(free_.size()); }
  int num_blocks() const { return n_; }
  // Prefix-cache membership: a cached page whose only reference is the cache's is
  // evictable; the count is kept up to date on every refcount transition (O(1)).
  void set_cached(int b, bool cached);
  int num_evictable() const { return n_evictable_; }

 private:
  int n_;
  std::vector<int> free_;
  std::vector<int> ref_;
  std::vector<uint8_t> cached_;
  int n_evictable_ = 0;
};

struct RadixNode {
  int block = -1;
  std::vector<int32_t> key;  // the page's tokens (block_size of them)
  RadixNode* parent = nullptr;
  std::unordered_map<uint64_t, std::vector<std::unique_ptr<RadixNode>>> children;
  uint64_t last_access = 0;
  size_t num_children() const;
};

struct PrefixCacheStats {
  int64_t entries = 0;        // cached pages
  int64_t hit_tokens = 0;     // tokens served from cache
  int64_t miss_tokens = 0;    // tokens looked up but not cached
  int64_t hit_count = 0;      // lookups with >= 1 page hit
  int64_t miss_count = 0;     // lookups with 0 page hits
  int64_t eviction_count = 0; // pages evicted
};

class PrefixCache {
 public:
  PrefixCache(BlockAllocator* alloc, int block_size, int max_cached_blocks);

  // Longest cached page-aligned prefix of tokens[0:max_tokens). Returns the
  // page ids (NOT incref'd) and touches the path. Counts a hit/miss.
  std::vector<int> match(const int32_t* tokens, int n_tokens, int max_tokens, bool count = true);
  // hit/miss accounting of one lookup, for callers that count only once the
  // lookup's result is actually used (scheduler admission can fail and retry)
  void record_lookup(int n_tokens, int hit_pages);
  // Insert the first n_full_pages pages of (tokens, blocks). The cache takes a
  // reference on every page it newly stores. Returns #pages newly cached.
  int insert(const int32_t* tokens, int n_tokens, const int* blocks, int n_blocks);
  // Evict up to n pages that only the cache references (LRU leaves first).
  int evict(int n);
  // Pages evictable right now (cache-only references).
  int evictable() const;
  void clear();  // drop every page (hot-swap / reset)

  int block_size() const { return bs_; }
  int max_cached_blocks() const { return max_cached_; }
  void set_max_cached_blocks(int m) { max_cached_ = m; }
  const PrefixCacheStats& stats() const { return stats_; }
  void reset_stats();
  // Last access tick of the node holding page `block` (0 if not cached).
  uint64_t last_access_of(int block) const;
  uint64_t tick() const { return tick_; }

 private:
  static uint64_t hash_page(const int32_t* t, int n);
  RadixNode* find_child(RadixNode* n, const int32_t* t) const;
  void remove_leaf(RadixNode* leaf);
  void enforce_limit();
  void touch(RadixNode* n);  // last_access = tick_, keeping the leaf index ordered

  BlockAllocator* alloc_;
  int bs_;
  int max_cached_;
  RadixNode root_;
  uint64_t tick_ = 0;
  PrefixCacheStats stats_;
  std::unordered_map<int, RadixNode*> by_block_;
  // every leaf ordered by (last_access, node): LRU eviction walks it from the front,
  // skipping leaves still referenced by a sequence (at most one tail page per live
  // sequence), so eviction costs O(log n) per page instead of a whole-tree walk
  std::set<std::pair<uint64_t, RadixNode*>> leaves_;
};

}  // namespace xgs
