// Native host runtime core: tokenizer trie and paged-KV block manager (no Python dependency).
//
// native.cpp binds these classes to Python (pybind11 module `_native`); tests/native/
// test_runtime.cpp drives them directly in a standalone binary built with
// -fsanitize=address,undefined (host-side C++ under ASan/UBSan in CPU tests).
#pragma once

#include <cstdint>
#include <algorithm>
#include <deque>
#include <iterator>
#include <list>
#include <stdexcept>
#include <string>
#include <tuple>
#include <unordered_map>
#include <utility>
#include <vector>

namespace ka {

// ------------------------------------------------------------------------------------------------
class Trie {
 public:
  // sparse edges: one hash map keyed by (node << 8 | byte); ~10^6 edges for a 128k vocabulary
  Trie() { ids_.push_back(-1); }

  void add(const std::string& bytes, int id) {
    uint32_t n = 0;
    for (unsigned char c : bytes) {
      const uint64_t key = ((uint64_t)n << 8) | c;
      auto it = edges_.find(key);
      if (it == edges_.end()) {
        const uint32_t nxt = (uint32_t)ids_.size();
        ids_.push_back(-1);
        edges_.emplace(key, nxt);
        n = nxt;
      } else {
        n = it->second;
      }
    }
    ids_[n] = id;
  }

  std::vector<int> encode(const std::string& data) const {
    std::vector<int> out;
    out.reserve(data.size() / 3 + 4);
    const size_t n = data.size();
    size_t i = 0;
    while (i < n) {
      uint32_t node = 0;
      int best = -1;
      size_t best_len = 0, j = i;
      while (j < n) {
        auto it = edges_.find(((uint64_t)node << 8) | (unsigned char)data[j]);
        if (it == edges_.end()) break;
        node = it->second;
        ++j;
        if (ids_[node] >= 0) {
          best = ids_[node];
          best_len = j - i;
        }
      }
      if (best < 0) throw std::runtime_error("byte not covered by the vocabulary");
      out.push_back(best);
      i += best_len;
    }
    return out;
  }

  size_t size() const { return ids_.size(); }

 private:
  std::unordered_map<uint64_t, uint32_t> edges_;
  std::vector<int> ids_;
};

// ------------------------------------------------------------------------------------------------
static inline uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x += 0x9e3779b97f4a7c15ULL;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

class BlockManager {
 public:
  BlockManager(int num_blocks, int block_size, bool prefix_caching)
      : num_blocks_(num_blocks), bs_(block_size), prefix_(prefix_caching), ref_(num_blocks, 0),
        hash_(num_blocks, 0), has_hash_(num_blocks, 0), lru_pos_(num_blocks), parent_(num_blocks, 0),
        btoks_(num_blocks) {
    for (int b = 0; b < num_blocks; ++b) free_.push_back(b);
  }

  static uint64_t chain_hash(uint64_t parent, const std::vector<int>& toks, size_t begin, size_t end) {
    uint64_t h = mix64(parent ^ 0x51ed270b27c3f2a5ULL);
    for (size_t i = begin; i < end; ++i) h = mix64(h ^ (uint64_t)(uint32_t)toks[i]);
    return h;
  }

  int num_free() const { return (int)(free_.size() + lru_.size()); }
  int num_used() const { return num_blocks_ - num_free(); }
  int blocks_needed(int ntok) const { return (ntok + bs_ - 1) / bs_; }

  // returns (table, cached_tokens, hashes)
  std::tuple<std::vector<int>, int, std::vector<uint64_t>> allocate_prompt(const std::vector<int>& toks) {
    std::vector<int> table;
    std::vector<uint64_t> hashes;
    int cached = 0;
    uint64_t parent = 0;
    const int n_full = prefix_ ? ((int)toks.size() - 1) / bs_ : 0;
    ++queries_;
    for (int i = 0; i < n_full; ++i) {
      const uint64_t h = chain_hash(parent, toks, (size_t)i * bs_, (size_t)(i + 1) * bs_);
      auto it = cached_.find(h);
      if (it == cached_.end()) break;
      acquire(it->second);
      table.push_back(it->second);
      hashes.push_back(h);
      parent = h;
      cached += bs_;
    }
    if (cached) ++hits_;
    const int need = blocks_needed((int)toks.size()) - (int)table.size();
    if (need > num_free()) {
      for (int b : table) release(b);
      throw std::runtime_error("NoFreeBlocks");
    }
    for (int k = 0; k < need; ++k) {
      const int b = pop_free();
      acquire(b);
      table.push_back(b);
    }
    return {table, cached, hashes};
  }

  std::vector<uint64_t> register_computed(const std::vector<int>& table, const std::vector<int>& toks,
                                          std::vector<uint64_t> hashes) {
    if (!prefix_) return hashes;
    uint64_t parent = hashes.empty() ? 0 : hashes.back();
    const int n_full = (int)toks.size() / bs_;
    for (int i = (int)hashes.size(); i < n_full; ++i) {
      const uint64_t h = chain_hash(parent, toks, (size_t)i * bs_, (size_t)(i + 1) * bs_);
      const int b = table[i];
      hashes.push_back(h);
      parent = h;
      if (cached_.find(h) == cached_.end() && !has_hash_[b]) {
        cached_[h] = b;
        hash_[b] = h;
        has_hash_[b] = 1;
        const uint64_t par = i > 0 ? hashes[i - 1] : 0;
        parent_[b] = par;
        btoks_[b].assign(toks.begin() + (size_t)i * bs_, toks.begin() + (size_t)(i + 1) * bs_);
        auto& kids = children_[par];
        if (kids.size() >= 4) kids.erase(kids.begin());
        kids.push_back(b);
      }
    }
    return hashes;
  }

  // sub-block reuse (engine/block_manager.py reuse_partial): returns (src, r) or (-1, 0)
  std::pair<int, int> reuse_partial(const std::vector<int>& toks, int cached, const std::vector<uint64_t>& hashes) {
    if (!prefix_) return {-1, 0};
    const int maxr = std::min(bs_, (int)toks.size() - 1 - cached);
    if (maxr <= 0) return {-1, 0};
    const uint64_t par = hashes.empty() ? 0 : hashes.back();
    auto it = children_.find(par);
    if (it == children_.end()) return {-1, 0};
    int best = -1, best_r = 0;
    for (int b : it->second) {
      if (!has_hash_[b] || parent_[b] != par) continue;
      int r = 0;
      while (r < maxr && btoks_[b][r] == toks[cached + r]) ++r;
      if (r > best_r) { best = b; best_r = r; }
    }
    if (best_r == 0) return {-1, 0};
    acquire(best);
    partial_ += best_r;
    return {best, best_r};
  }

  void unpin(int b) { release(b); }
  long partial_tokens() const { return partial_; }

  std::vector<int> ensure_capacity(std::vector<int> table, int ntok) {
    // all-or-nothing: a partial grow would leak the blocks taken before the failure (the caller
    // only sees the returned table)
    if (blocks_needed(ntok) - (int)table.size() > num_free()) throw std::runtime_error("NoFreeBlocks");
    while ((int)table.size() * bs_ < ntok) {
      const int b = pop_free();
      acquire(b);
      table.push_back(b);
    }
    return table;
  }

  void free_table(const std::vector<int>& table) {
    for (int b : table) release(b);
  }

  void reset_prefix_cache() {
    for (int b : lru_) {
      unhash(b);
      free_.push_back(b);
    }
    lru_.clear();
    in_lru_.clear();
    for (auto it = cached_.begin(); it != cached_.end();) {
      if (ref_[it->second] > 0) ++it;
      else it = cached_.erase(it);
    }
  }

  int ref(int b) const { return ref_.at(b); }
  size_t num_index_keys() const { return children_.size(); }
  long hits() const { return hits_; }
  long queries() const { return queries_; }

 private:
  int pop_free() {
    if (!free_.empty()) {
      const int b = free_.front();
      free_.pop_front();
      return b;
    }
    if (!lru_.empty()) {
      const int b = lru_.front();
      lru_.pop_front();
      in_lru_.erase(b);
      if (has_hash_[b]) {
        auto it = cached_.find(hash_[b]);
        if (it != cached_.end() && it->second == b) cached_.erase(it);
      }
      unhash(b);
      return b;
    }
    throw std::runtime_error("NoFreeBlocks");
  }

  void acquire(int b) {
    if (ref_[b] == 0) {
      auto it = in_lru_.find(b);
      if (it != in_lru_.end()) {
        lru_.erase(lru_pos_[b]);
        in_lru_.erase(it);
      }
    }
    ++ref_[b];
  }

  void release(int b) {
    if (--ref_[b] < 0) throw std::runtime_error("block refcount underflow");
    if (ref_[b] == 0) {
      auto it = has_hash_[b] ? cached_.find(hash_[b]) : cached_.end();
      if (it != cached_.end() && it->second == b) {
        lru_.push_back(b);
        lru_pos_[b] = std::prev(lru_.end());
        in_lru_[b] = 1;
      } else {
        unhash(b);
        free_.push_back(b);
      }
    }
  }

  // A block that leaves the prefix cache also leaves its parent's sibling index, so the index
  // holds only published blocks and its key count stays bounded by the cache size (one key per
  // parent with a live child) however many distinct prompts pass through.
  void unhash(int b) {
    if (!has_hash_[b]) return;
    has_hash_[b] = 0;
    auto it = children_.find(parent_[b]);
    if (it != children_.end()) {
      auto& kids = it->second;
      kids.erase(std::remove(kids.begin(), kids.end(), b), kids.end());
      if (kids.empty()) children_.erase(it);
    }
    btoks_[b].clear();
  }

  int num_blocks_, bs_;
  bool prefix_;
  std::vector<int> ref_;
  std::vector<uint64_t> hash_;
  std::vector<char> has_hash_;
  std::deque<int> free_;
  std::list<int> lru_;
  std::vector<std::list<int>::iterator> lru_pos_;
  std::unordered_map<int, char> in_lru_;
  std::unordered_map<uint64_t, int> cached_;
  std::vector<uint64_t> parent_;                           // parent hash of a published block
  std::vector<std::vector<int>> btoks_;                    // its tokens (sub-block reuse)
  std::unordered_map<uint64_t, std::vector<int>> children_;  // parent hash -> up to 4 recent children
  long hits_ = 0, queries_ = 0, partial_ = 0;
};

}  // namespace ka
