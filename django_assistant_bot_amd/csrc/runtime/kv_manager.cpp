#include "kv_manager.h"

#include <algorithm>
#include <functional>
#include <iterator>
#include <stdexcept>

namespace dab {

KVBlockManager::KVBlockManager(int num_blocks, int block_size, bool prefix_cache)
    : num_blocks_(num_blocks), block_size_(block_size), prefix_cache_(prefix_cache) {
  if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("num_blocks and block_size must be > 0");
  free_.reserve(num_blocks);
  for (int b = 0; b < num_blocks; ++b) free_.push_back(b);  // ascending = a valid min-heap
  lru_cap_ = std::max(64, num_blocks / 4);
  ref_.assign(num_blocks, 0);
  block_hash_.assign(num_blocks, 0);
  lru_pos_.resize(num_blocks);
  in_lru_.assign(num_blocks, 0);
}

uint64_t KVBlockManager::chain_hash(uint64_t parent, const int32_t* toks, int n) const {
  uint64_t h = parent ^ 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < n; ++i) {
    h ^= (uint64_t)(uint32_t)toks[i] + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 0x100000001B3ull;
  }
  return h ? h : 1;  // 0 is reserved for "unregistered"
}

int32_t KVBlockManager::alloc_block() {
  int32_t b;
  if (!free_.empty()) {
    std::pop_heap(free_.begin(), free_.end(), std::greater<int32_t>());
    b = free_.back();
    free_.pop_back();
  } else if (!lru_.empty()) {
    b = lru_.front();
    lru_.pop_front();
    in_lru_[b] = 0;
    cached_.erase(block_hash_[b]);
    block_hash_[b] = 0;
  } else {
    return -1;
  }
  ref_[b] = 1;
  return b;
}

void KVBlockManager::release_block(int32_t b) {
  if (--ref_[b] > 0) return;
  if (prefix_cache_ && block_hash_[b] != 0) {
    lru_.push_back(b);
    lru_pos_[b] = std::prev(lru_.end());
    in_lru_[b] = 1;
    if ((int)lru_.size() > lru_cap_) {  // the oldest cached prefix block goes back to the free heap
      const int32_t e = lru_.front();
      lru_.pop_front();
      in_lru_[e] = 0;
      cached_.erase(block_hash_[e]);
      block_hash_[e] = 0;
      push_free(e);
    }
  } else {
    block_hash_[b] = 0;
    push_free(b);
  }
}

void KVBlockManager::push_free(int32_t b) {
  free_.push_back(b);
  std::push_heap(free_.begin(), free_.end(), std::greater<int32_t>());
}

int KVBlockManager::add_sequence(int64_t seq_id, const std::vector<int32_t>& tokens, int reserve) {
  if (seqs_.count(seq_id)) throw std::invalid_argument("sequence already registered");
  const int n = (int)tokens.size();
  const int need_tokens = n + (reserve > 0 ? reserve : 0);
  const int need_blocks = (need_tokens + block_size_ - 1) / block_size_;
  // prefix lookup: at most (n - 1) tokens may come from the cache, so prefill computes >= 1 token
  std::vector<int32_t> hit_blocks;
  std::vector<uint64_t> hit_hashes;
  if (prefix_cache_ && n > 1) {
    const int max_full = (n - 1) / block_size_;
    uint64_t h = 0;
    for (int i = 0; i < max_full; ++i) {
      h = chain_hash(h, tokens.data() + (size_t)i * block_size_, block_size_);
      auto it = cached_.find(h);
      if (it == cached_.end()) break;
      hit_blocks.push_back(it->second);
      hit_hashes.push_back(h);
    }
  }
  // availability: blocks reused from the LRU are not free capacity for the remainder
  int reused_from_lru = 0;
  for (int32_t b : hit_blocks) reused_from_lru += in_lru_[b] ? 1 : 0;
  const int fresh = need_blocks - (int)hit_blocks.size();
  if (fresh > num_free_blocks() - reused_from_lru) return -1;
  Seq s;
  for (int32_t b : hit_blocks) {
    if (in_lru_[b]) {
      lru_.erase(lru_pos_[b]);
      in_lru_[b] = 0;
    }
    ++ref_[b];
    s.blocks.push_back(b);
  }
  s.hashes = hit_hashes;
  for (int i = 0; i < fresh; ++i) s.blocks.push_back(alloc_block());
  s.tokens = tokens;
  const int cached_tokens = (int)hit_blocks.size() * block_size_;
  prefix_hits_ += cached_tokens;
  seqs_.emplace(seq_id, std::move(s));
  return cached_tokens;
}

bool KVBlockManager::extend(int64_t seq_id, int n) {
  auto it = seqs_.find(seq_id);
  if (it == seqs_.end()) throw std::invalid_argument("unknown sequence");
  Seq& s = it->second;
  const int need = (int)s.tokens.size() + n;
  const int need_blocks = (need + block_size_ - 1) / block_size_;
  const int more = need_blocks - (int)s.blocks.size();
  if (more <= 0) return true;
  if (more > num_free_blocks()) return false;
  for (int i = 0; i < more; ++i) s.blocks.push_back(alloc_block());
  return true;
}

void KVBlockManager::append_tokens(int64_t seq_id, const std::vector<int32_t>& tokens) {
  auto it = seqs_.find(seq_id);
  if (it == seqs_.end()) throw std::invalid_argument("unknown sequence");
  Seq& s = it->second;
  s.tokens.insert(s.tokens.end(), tokens.begin(), tokens.end());
  if ((int)s.tokens.size() > (int)s.blocks.size() * block_size_) throw std::runtime_error("KV capacity exceeded");
}

void KVBlockManager::commit_prefix(int64_t seq_id, int n_computed) {
  if (!prefix_cache_) return;
  auto it = seqs_.find(seq_id);
  if (it == seqs_.end()) return;
  Seq& s = it->second;
  const int full = std::min<int>(n_computed, (int)s.tokens.size()) / block_size_;
  uint64_t h = s.hashes.empty() ? 0 : s.hashes.back();
  for (int i = (int)s.hashes.size(); i < full && i < (int)s.blocks.size(); ++i) {
    h = chain_hash(h, s.tokens.data() + (size_t)i * block_size_, block_size_);
    s.hashes.push_back(h);
    const int32_t b = s.blocks[i];
    if (block_hash_[b] == 0 && !cached_.count(h)) {
      block_hash_[b] = h;
      cached_[h] = b;
    }
  }
}

void KVBlockManager::free_sequence(int64_t seq_id) {
  auto it = seqs_.find(seq_id);
  if (it == seqs_.end()) return;
  for (int32_t b : it->second.blocks) release_block(b);
  seqs_.erase(it);
}

int KVBlockManager::num_tokens(int64_t seq_id) const {
  auto it = seqs_.find(seq_id);
  return it == seqs_.end() ? 0 : (int)it->second.tokens.size();
}

int KVBlockManager::capacity_tokens(int64_t seq_id) const {
  auto it = seqs_.find(seq_id);
  return it == seqs_.end() ? 0 : (int)it->second.blocks.size() * block_size_;
}

const std::vector<int32_t>& KVBlockManager::blocks(int64_t seq_id) const {
  auto it = seqs_.find(seq_id);
  if (it == seqs_.end()) throw std::invalid_argument("unknown sequence");
  return it->second.blocks;
}

void KVBlockManager::slot_mapping(int64_t seq_id, int start, int n, int64_t* out) const {
  const auto& bl = blocks(seq_id);
  for (int i = 0; i < n; ++i) {
    const int pos = start + i;
    const int bi = pos / block_size_;
    if (bi >= (int)bl.size()) throw std::out_of_range("slot beyond allocated blocks");
    out[i] = (int64_t)bl[bi] * block_size_ + (pos % block_size_);
  }
}

int KVBlockManager::prepare_decode(const std::vector<int64_t>& seq_ids, const std::vector<int32_t>& tokens,
                                   int max_blocks, int32_t* ids, int32_t* pos, int64_t* slots, int32_t* ctx,
                                   int32_t* block_table) {
  if (seq_ids.size() != tokens.size()) throw std::invalid_argument("seq_ids / tokens length mismatch");
  for (size_t i = 0; i < seq_ids.size(); ++i)
    if (!extend(seq_ids[i], 1)) return (int)i;
  for (size_t i = 0; i < seq_ids.size(); ++i) {
    Seq& s = seqs_.at(seq_ids[i]);
    s.tokens.push_back(tokens[i]);
    const int p = (int)s.tokens.size() - 1;
    ids[i] = tokens[i];
    pos[i] = p;
    slots[i] = (int64_t)s.blocks[p / block_size_] * block_size_ + (p % block_size_);
    ctx[i] = p + 1;
    if ((int)s.blocks.size() > max_blocks) throw std::out_of_range("block table wider than max_blocks");
    int32_t* row = block_table + i * (size_t)max_blocks;
    std::copy(s.blocks.begin(), s.blocks.end(), row);
    std::fill(row + s.blocks.size(), row + max_blocks, 0);
  }
  return -1;
}

void KVBlockManager::block_table(const std::vector<int64_t>& seq_ids, int max_blocks, int32_t* out) const {
  for (size_t r = 0; r < seq_ids.size(); ++r) {
    int32_t* row = out + r * max_blocks;
    int i = 0;
    if (seq_ids[r] >= 0) {
      const auto& bl = blocks(seq_ids[r]);
      if ((int)bl.size() > max_blocks) throw std::out_of_range("block table wider than max_blocks");
      for (; i < (int)bl.size(); ++i) row[i] = bl[i];
    }
    for (; i < max_blocks; ++i) row[i] = 0;
  }
}

}  // namespace dab
