// Paged KV-cache block pool with hash-chained prefix caching and LRU eviction —
// pybind-free core shared by the Python binding (block_pool.cpp) and the
// sanitizer stress test (csrc/tests/runtime_stress.cpp).
//
// Reference parity: the reference's HF-tier engine sizes a paged KV cache from
// `--gpu-memory-utilization 0.90` (vllm-models/helm-chart/templates/
// model-deployments.yaml:35-36); this is our allocator for that pool.
#pragma once

#include <cstdint>
#include <cstring>
#include <list>
#include <stdexcept>
#include <unordered_map>
#include <utility>
#include <vector>

namespace hipserve_rt {

inline uint64_t mix64(uint64_t x) {
  x ^= x >> 31; x *= 0x7FB5D329728EA185ull;
  x ^= x >> 27; x *= 0x81DADEF4BC2DD44Dull;
  x ^= x >> 33;
  return x;
}

class BlockPool {
 public:
  BlockPool(int num_blocks, int block_size, bool prefix_caching)
      : num_blocks_(num_blocks), block_size_(block_size), prefix_(prefix_caching),
        ref_(num_blocks, 0), hash_(num_blocks, 0), has_hash_(num_blocks, 0),
        lru_pos_(num_blocks) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("bad pool size");
    free_.reserve(num_blocks);
    for (int i = num_blocks - 1; i >= 0; --i) free_.push_back(i);
    tokens_.resize((size_t)num_blocks * block_size, -1);
  }

  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  // blocks that can be handed out right now (free + cached-but-unreferenced)
  int num_free() const { return (int)free_.size() + (int)lru_.size(); }
  int num_cached() const { return (int)cache_.size(); }
  double usage() const { return 1.0 - (double)num_free() / num_blocks_; }

  std::vector<int> allocate(int n) {
    if (n > num_free()) throw std::runtime_error("KV cache out of blocks");
    std::vector<int> out;
    out.reserve(n);
    for (int i = 0; i < n; ++i) {
      int b;
      if (!free_.empty()) {
        b = free_.back();
        free_.pop_back();
      } else {  // evict least-recently-freed cached block
        b = lru_.front();
        lru_.pop_front();
        drop_hash(b);
      }
      ref_[b] = 1;
      out.push_back(b);
    }
    return out;
  }

  void free(const std::vector<int>& ids) {
    // free in reverse so the tail of a sequence (least shareable) is evicted first
    for (auto it = ids.rbegin(); it != ids.rend(); ++it) {
      const int b = *it;
      if (b < 0 || b >= num_blocks_ || ref_[b] <= 0) throw std::runtime_error("double free of KV block");
      if (--ref_[b] == 0) {
        if (has_hash_[b]) {
          lru_.push_back(b);
          lru_pos_[b] = std::prev(lru_.end());
        } else {
          free_.push_back(b);
        }
      }
    }
  }

  uint64_t block_hash(uint64_t parent, const std::vector<int>& toks) const {
    uint64_t h = mix64(parent ^ 0x9E3779B97F4A7C15ull);
    for (int t : toks) h = mix64(h ^ ((uint64_t)(uint32_t)t + 0x632BE59BD9B4E019ull));
    return h;
  }

  // Longest cached prefix of `tokens` in whole blocks; returned blocks are
  // referenced (caller owns them). Leaves at least one token uncomputed so the
  // model still produces logits for the last prompt token.
  std::pair<std::vector<int>, int> match_prefix(const std::vector<int>& tokens) {
    std::vector<int> hit;
    if (!prefix_) return {hit, 0};
    const int full = ((int)tokens.size() - 1) / block_size_;
    uint64_t parent = 0;
    std::vector<int> blk(block_size_);
    for (int i = 0; i < full; ++i) {
      std::memcpy(blk.data(), tokens.data() + (size_t)i * block_size_, block_size_ * sizeof(int));
      const uint64_t h = block_hash(parent, blk);
      auto it = cache_.find(h);
      if (it == cache_.end()) break;
      const int b = it->second;
      if (std::memcmp(&tokens_[(size_t)b * block_size_], blk.data(), block_size_ * sizeof(int)) != 0) break;
      if (ref_[b] == 0) {  // revive from the evictable LRU
        lru_.erase(lru_pos_[b]);
      }
      ++ref_[b];
      hit.push_back(b);
      parent = h;
    }
    const int ntok = (int)hit.size() * block_size_;
    return {hit, ntok};
  }

  // Register the full blocks [first, last) of a sequence whose tokens are known.
  void register_full_blocks(const std::vector<int>& block_ids, const std::vector<int>& tokens,
                            int first, int last) {
    if (!prefix_) return;
    uint64_t parent = 0;
    std::vector<int> blk(block_size_);
    for (int i = 0; i < last && i < (int)block_ids.size(); ++i) {
      if ((size_t)(i + 1) * block_size_ > tokens.size()) break;
      std::memcpy(blk.data(), tokens.data() + (size_t)i * block_size_, block_size_ * sizeof(int));
      const uint64_t h = block_hash(parent, blk);
      parent = h;
      if (i < first) continue;
      const int b = block_ids[i];
      if (has_hash_[b]) continue;
      if (cache_.count(h)) continue;  // an identical block is already cached
      cache_[h] = b;
      hash_[b] = h;
      has_hash_[b] = 1;
      std::memcpy(&tokens_[(size_t)b * block_size_], blk.data(), block_size_ * sizeof(int));
    }
  }

  // Incremental form: `tokens` holds ONLY blocks [first, last) and `parent` is the
  // chained hash of block first-1 (0 for the first block); returns the hash of
  // block last-1, for the next call. O(new tokens) instead of O(context).
  uint64_t register_blocks(const std::vector<int>& block_ids, const std::vector<int>& tokens, int first,
                           int last, uint64_t parent) {
    std::vector<int> blk(block_size_);
    for (int i = first; i < last && i < (int)block_ids.size(); ++i) {
      const size_t off = (size_t)(i - first) * block_size_;
      if (off + block_size_ > tokens.size()) break;
      std::memcpy(blk.data(), tokens.data() + off, block_size_ * sizeof(int));
      const uint64_t h = block_hash(parent, blk);
      parent = h;
      if (!prefix_) continue;
      const int b = block_ids[i];
      if (has_hash_[b] || cache_.count(h)) continue;
      cache_[h] = b;
      hash_[b] = h;
      has_hash_[b] = 1;
      std::memcpy(&tokens_[(size_t)b * block_size_], blk.data(), block_size_ * sizeof(int));
    }
    return parent;
  }

  void reset_prefix_cache() {
    for (int b : lru_) { drop_hash(b); free_.push_back(b); }
    lru_.clear();
    for (int b = 0; b < num_blocks_; ++b) if (has_hash_[b]) drop_hash(b);
  }

  int refcount(int b) const { return ref_.at(b); }

 private:
  void drop_hash(int b) {
    if (!has_hash_[b]) return;
    auto it = cache_.find(hash_[b]);
    if (it != cache_.end() && it->second == b) cache_.erase(it);
    has_hash_[b] = 0;
  }

  int num_blocks_, block_size_;
  bool prefix_;
  std::vector<int> free_;
  std::vector<int> ref_;
  std::vector<uint64_t> hash_;
  std::vector<char> has_hash_;
  std::list<int> lru_;
  std::vector<std::list<int>::iterator> lru_pos_;
  std::unordered_map<uint64_t, int> cache_;
  std::vector<int> tokens_;
};

}  // namespace hipserve_rt
