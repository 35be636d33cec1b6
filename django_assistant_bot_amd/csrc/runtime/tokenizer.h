// Offline, deterministic word-hash tokenizer (native, multi-threaded batch encode).
//
// The reference loads HF tokenizers from the hub (ai/embedders/transformers.py:11-12,
// ai/providers/transformers.py:18-19).  This build has no network and benchmarks random-init
// weights, so the engine ships its own tokenizer with the same contract (special tokens, truncation
// to the model's max length, [CLS] ... [SEP] framing for encoders, BOS for decoders).  Real HF
// `tokenizer.json` files are used instead when present (python side, tokenizers library).
//
// Normalisation: lower-case ASCII and Cyrillic, split on whitespace, every punctuation / symbol
// code point is its own token.  A word maps to  first_id + fnv1a64(word) % (last_id - first_id).
// Decoding inverts ids seen during encoding; unseen ids (e.g. sampled by a random-init model)
// decode to a deterministic pronounceable pseudo-word so generated text is still text.
#pragma once
#include <cstdint>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace dab {

struct TokenizerConfig {
  int vocab_size = 30522;
  int first_id = 1000;    // first hashed id
  int last_id = 30522;    // one past the last hashed id
  int pad_id = 0;
  int unk_id = 100;
  int cls_id = 101;       // encoder framing (or BOS for decoders when sep_id < 0)
  int sep_id = 102;       // < 0: no trailing separator (decoder mode)
  int max_word_chars = 24;  // longer words are split into pieces of this many code points
};

class HashTokenizer {
 public:
  explicit HashTokenizer(const TokenizerConfig& cfg) : cfg_(cfg) {}

  // Raw word-piece ids, no framing.
  std::vector<int32_t> encode_raw(const std::string& text, bool remember = true) const;
  // Framed + truncated to max_len (0 = unlimited).
  std::vector<int32_t> encode(const std::string& text, bool add_special, int max_len) const;
  // Batch encode on `threads` worker threads; returns flat ids and offsets (size n+1).
  void encode_batch(const std::vector<std::string>& texts, bool add_special, int max_len, int threads,
                    std::vector<int32_t>& ids, std::vector<int64_t>& offsets) const;
  std::string decode(const std::vector<int32_t>& ids, bool skip_special) const;
  // The bytes each id adds to decode() output after a first token (" word" or a lone punctuation
  // character; "" for special ids): the vocabulary of the JSON-constrained decoder.
  std::vector<std::string> token_texts() const;
  // Number of whitespace separated words (used by the reference's crude token estimate).
  static int64_t count_words(const std::string& text);
  const TokenizerConfig& config() const { return cfg_; }

 private:
  TokenizerConfig cfg_;
  mutable std::mutex mu_;
  mutable std::unordered_map<int32_t, std::string> seen_;
  int32_t word_id(const std::string& w) const;
  std::string pseudo_word(int32_t id) const;
  // Framed + truncated ids of one text into ``out``; words whose id is not yet marked in ``mark``
  // (one byte per vocabulary id, owned by the calling thread) are appended to ``fresh``.
  void encode_into(const std::string& text, bool add_special, int max_len, std::vector<int32_t>& out,
                   std::vector<uint8_t>& mark, std::vector<std::pair<int32_t, std::string>>& fresh) const;
  void remember(std::vector<std::pair<int32_t, std::string>>& fresh) const;
};

}  // namespace dab
