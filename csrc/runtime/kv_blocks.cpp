#include "kv_blocks.h"

#include <algorithm>
#include <cstring>
#include <queue>
#include <stdexcept>

namespace xgs {

// ---------------------------------------------------------------------------
// BlockAllocator
// ---------------------------------------------------------------------------
BlockAllocator::BlockAllocator(int num_blocks) : n_(num_blocks), ref_(num_blocks, 0), cached_(num_blocks, 0) {
  free_.reserve(num_blocks);
  // Pop order ascending page id: keeps early pages (and their TLB entries) hot.
  for (int i = num_blocks - 1; i >= 0; --i) free_.push_back(i);
}

int BlockAllocator::alloc() {
  if (free_.empty()) return -1;
  int b = free_.back();
  free_.pop_back();
  ref_[b] = 1;
  return b;
}

void BlockAllocator::incref(int b) {
  if (b < 0 || b >= n_ || ref_[b] <= 0) throw std::runtime_error("incref on a free page");
  if (cached_[b] && ref_[b] == 1) --n_evictable_;
  ++ref_[b];
}

void BlockAllocator::decref(int b) {
  if (b < 0 || b >= n_ || ref_[b] <= 0) throw std::runtime_error("decref on a free page");
  if (--ref_[b] == 0) free_.push_back(b);
  else if (cached_[b] && ref_[b] == 1) ++n_evictable_;
}

void BlockAllocator::set_cached(int b, bool cached) {
  if (b < 0 || b >= n_ || ref_[b] <= 0) throw std::runtime_error("set_cached on a free page");
  if (cached == static_cast<bool>(cached_[b])) return;
  cached_[b] = cached ? 1 : 0;
  if (ref_[b] == 1) n_evictable_ += cached ? 1 : -1;
}

// ---------------------------------------------------------------------------
// PrefixCache
// ---------------------------------------------------------------------------
size_t RadixNode::num_children() const {
  size_t n = 0;
  for (const auto& kv : children) n += kv.second.size();
  return n;
}

PrefixCache::PrefixCache(BlockAllocator* alloc, int block_size, int max_cached_blocks)
    : alloc_(alloc), bs_(block_size), max_cached_(max_cached_blocks) {}

uint64_t PrefixCache::hash_page(const int32_t* t, int n) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a over the 32-bit token ids
  for (int i = 0; i < n; ++i) {
    uint32_t v = static_cast<uint32_t>(t[i]);
    for (int k = 0; k < 4; ++k) {
      h ^= (v >> (8 * k)) & 0xFF;
      h *= 1099511628211ull;
    }
  }
  return h;
}

RadixNode* PrefixCache::find_child(RadixNode* n, const int32_t* t) const {
  auto it = n->children.find(hash_page(t, bs_));
  if (it == n->children.end()) return nullptr;
  for (const auto& c : it->second)
    if (std::memcmp(c->key.data(), t, sizeof(int32_t) * bs_) == 0) return c.get();
  return nullptr;
}

std::vector<int> PrefixCache::match(const int32_t* tokens, int n_tokens, int max_tokens, bool count) {
  std::vector<int> out;
  int lim = std::min(n_tokens, max_tokens);
  int pages = lim / bs_;
  RadixNode* cur = &root_;
  ++tick_;
  for (int p = 0; p < pages; ++p) {
    RadixNode* c = find_child(cur, tokens + p * bs_);
    if (!c) break;
    touch(c);
    out.push_back(c->block);
    cur = c;
  }
  if (count) record_lookup(n_tokens, static_cast<int>(out.size()));
  return out;
}

void PrefixCache::record_lookup(int n_tokens, int hit_pages) {
  int hit = hit_pages * bs_;
  stats_.hit_tokens += hit;
  stats_.miss_tokens += std::max(0, n_tokens - hit);
  if (hit_pages == 0) ++stats_.miss_count; else ++stats_.hit_count;
}

int PrefixCache::insert(const int32_t* tokens, int n_tokens, const int* blocks, int n_blocks) {
  int pages = std::min(n_tokens / bs_, n_blocks);
  RadixNode* cur = &root_;
  int added = 0;
  ++tick_;
  for (int p = 0; p < pages; ++p) {
    const int32_t* t = tokens + p * bs_;
    RadixNode* c = find_child(cur, t);
    if (!c) {
      if (max_cached_ <= 0) break;
      auto node = std::make_unique<RadixNode>();
      node->block = blocks[p];
      node->key.assign(t, t + bs_);
      node->parent = cur;
      node->last_access = tick_;
      alloc_->incref(blocks[p]);
      alloc_->set_cached(blocks[p], true);
      c = node.get();
      by_block_[blocks[p]] = c;
      if (cur != &root_ && cur->children.empty()) leaves_.erase({cur->last_access, cur});  // no longer a leaf
      cur->children[hash_page(t, bs_)].push_back(std::move(node));
      leaves_.insert({c->last_access, c});
      ++stats_.entries;
      ++added;
    } else {
      touch(c);
    }
    cur = c;
  }
  enforce_limit();
  return added;
}

void PrefixCache::touch(RadixNode* n) {
  if (n->last_access == tick_) return;
  const bool leaf = n->children.empty();
  if (leaf) leaves_.erase({n->last_access, n});
  n->last_access = tick_;
  if (leaf) leaves_.insert({n->last_access, n});
}

void PrefixCache::remove_leaf(RadixNode* leaf) {
  RadixNode* par = leaf->parent;
  leaves_.erase({leaf->last_access, leaf});
  uint64_t h = hash_page(leaf->key.data(), bs_);
  auto it = par->children.find(h);
  auto& vec = it->second;
  int block = leaf->block;
  for (size_t i = 0; i < vec.size(); ++i) {
    if (vec[i].get() == leaf) {
      vec.erase(vec.begin() + i);  // destroys the node
      break;
    }
  }
  if (vec.empty()) par->children.erase(it);
  if (par != &root_ && par->children.empty()) leaves_.insert({par->last_access, par});  // became a leaf
  by_block_.erase(block);
  alloc_->set_cached(block, false);
  alloc_->decref(block);
  --stats_.entries;
  ++stats_.eviction_count;
}

int PrefixCache::evict(int n) {
  // oldest leaves first; a parent that becomes a leaf joins the index at its own
  // (older or newer) access time, so sweep again while a pass made progress
  int done = 0;
  bool progress = true;
  while (done < n && progress) {
    progress = false;
    for (auto it = leaves_.begin(); done < n && it != leaves_.end();) {
      RadixNode* l = it->second;
      if (alloc_->refcount(l->block) != 1) {  // still used by a live sequence
        ++it;
        continue;
      }
      ++it;  // remove_leaf erases l (and may insert its parent) -- advance first
      const uint64_t next_key = it != leaves_.end() ? it->first : UINT64_MAX;
      RadixNode* next_node = it != leaves_.end() ? it->second : nullptr;
      remove_leaf(l);
      ++done;
      progress = true;
      it = next_node ? leaves_.find({next_key, next_node}) : leaves_.end();
    }
  }
  return done;
}

int PrefixCache::evictable() const { return alloc_->num_evictable(); }

void PrefixCache::enforce_limit() {
  int excess = static_cast<int>(stats_.entries) - max_cached_;
  if (excess > 0) evict(excess);
}

void PrefixCache::clear() {
  // Evict everything evictable; pages still used by live sequences stay
  // referenced by those sequences and are simply forgotten by the cache.
  std::vector<RadixNode*> all;
  std::vector<RadixNode*> stack{&root_};
  while (!stack.empty()) {
    RadixNode* n = stack.back();
    stack.pop_back();
    for (auto& kv : n->children)
      for (auto& c : kv.second) {
        all.push_back(c.get());
        stack.push_back(c.get());
      }
  }
  for (RadixNode* n : all) {
    alloc_->set_cached(n->block, false);
    alloc_->decref(n->block);
  }
  stats_.eviction_count += static_cast<int64_t>(all.size());
  leaves_.clear();
  root_.children.clear();
  by_block_.clear();
  stats_.entries = 0;
}

void PrefixCache::reset_stats() {
  int64_t e = stats_.entries;
  stats_ = PrefixCacheStats{};
  stats_.entries = e;
}

uint64_t PrefixCache::last_access_of(int block) const {
  auto it = by_block_.find(block);
  return it == by_block_.end() ? 0 : it->second->last_access;
}

}  // namespace xgs
