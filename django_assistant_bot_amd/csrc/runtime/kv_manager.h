// Paged KV-cache block manager with content-hashed prefix caching (native runtime).
//
// The reference relies on HF DynamicCache inside model.generate (ai/providers/transformers.py:57-66):
// one contiguous, per-request cache, batch = 1.  The engine instead keeps one pool of fixed-size
// KV blocks in HBM ([num_blocks, Hkv, block_size, D] per layer, sized from the 288 GB budget) and
// gives every running sequence a block table, which is what the paged decode / prefill attention
// kernels read.  Full prompt blocks are registered under a chained content hash so requests that
// share a prefix (the bot's system prompt, repeated questions) reuse the cached KV instead of
// re-running prefill; unreferenced cached blocks are evicted LRU when the free list is empty, and
// at most a quarter of the pool (>= 64 blocks) is kept as cached prefixes.  Free blocks are handed
// out lowest id first (a min-heap), so the live blocks of a batch stay packed at the low end of the
// pool: decode attention reads every live block each step, and scattered over an engine-sized pool
// (24k blocks) they streamed ~3 % slower than packed (profiles/decode_round2.md).
#pragma once
#include <cstdint>
#include <list>
#include <unordered_map>
#include <vector>

namespace dab {

class KVBlockManager {
 public:
  KVBlockManager(int num_blocks, int block_size, bool prefix_cache);

  // Admits a sequence: reuses cached prefix blocks, allocates blocks for len(tokens)+reserve.
  // Returns the number of prompt tokens whose KV is already cached, or -1 if blocks are short
  // (nothing is allocated in that case).
  int add_sequence(int64_t seq_id, const std::vector<int32_t>& tokens, int reserve);
  // Makes room for `n` more tokens at the end of the sequence; false if out of blocks.
  bool extend(int64_t seq_id, int n);
  // Appends generated token ids (kept for hashing / bookkeeping).
  void append_tokens(int64_t seq_id, const std::vector<int32_t>& tokens);
  // Registers the sequence's fully computed blocks among the first `n_computed` tokens.
  void commit_prefix(int64_t seq_id, int n_computed);
  void free_sequence(int64_t seq_id);

  bool has(int64_t seq_id) const { return seqs_.count(seq_id) != 0; }
  int num_tokens(int64_t seq_id) const;
  int capacity_tokens(int64_t seq_id) const;
  int num_free_blocks() const { return (int)free_.size() + (int)lru_.size(); }
  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  int64_t prefix_hits() const { return prefix_hits_; }
  const std::vector<int32_t>& blocks(int64_t seq_id) const;

  // One decode step for a batch: reserves one slot per sequence (returns the index of the first
  // sequence that cannot get a block, nothing appended then), else appends each sequence's last
  // token and fills ids / positions / slots / context lengths / block-table rows; returns -1.
  int prepare_decode(const std::vector<int64_t>& seq_ids, const std::vector<int32_t>& tokens, int max_blocks,
                     int32_t* ids, int32_t* pos, int64_t* slots, int32_t* ctx, int32_t* block_table);
  // slot ids (block * block_size + offset) of token positions [start, start + n)
  void slot_mapping(int64_t seq_id, int start, int n, int64_t* out) const;
  // block tables of several sequences into a [len(seq_ids), max_blocks] int32 matrix (-1 padding... 0)
  void block_table(const std::vector<int64_t>& seq_ids, int max_blocks, int32_t* out) const;

 private:
  struct Seq {
    std::vector<int32_t> blocks;
    std::vector<int32_t> tokens;
    std::vector<uint64_t> hashes;  // chained hash of each registered full block
  };
  int num_blocks_, block_size_;
  bool prefix_cache_;
  std::vector<int32_t> free_;  // min-heap (std::greater)
  int lru_cap_ = 64;
  std::vector<int32_t> ref_;
  std::vector<uint64_t> block_hash_;  // 0 = not registered
  std::unordered_map<uint64_t, int32_t> cached_;
  std::list<int32_t> lru_;  // registered blocks with ref == 0, least recent first
  std::vector<std::list<int32_t>::iterator> lru_pos_;
  std::vector<char> in_lru_;
  std::unordered_map<int64_t, Seq> seqs_;
  int64_t prefix_hits_ = 0;

  int32_t alloc_block();
  void push_free(int32_t b);
  void release_block(int32_t b);
  uint64_t chain_hash(uint64_t parent, const int32_t* toks, int n) const;
};

}  // namespace dab
