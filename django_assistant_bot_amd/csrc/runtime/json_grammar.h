// JSON-constrained decoding: a byte-level pushdown automaton for one JSON object, evaluated over a
// trie of the vocabulary's token byte strings, gives the set of tokens that keep the output a
// prefix of valid JSON -> an allowed-token bitmask per decode step (applied to the logits on the
// GPU before sampling, select.hip mask_logits).
//
// Replaces the reference's retry loop for JSON answers (assistant/bot/services/context_service/
// steps/classify.py:41-45, choose_known_question.py:45-50: up to 5 generations until json.loads
// succeeds): a constrained generation is valid JSON in one shot.
//
// Budget: every state has a shortest completion (the closing bytes it still needs, e.g. `"}]}`).
// A token is allowed only if the completion length after it fits in the tokens left after it
// (every completion byte is reachable with one single-byte token), so an answer cut by
// max_new_tokens still closes.  Nesting depth and whitespace runs are capped.
#pragma once
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace dab {

struct JsonState {
  uint8_t mode = 0;    // JsonMode
  uint8_t sub = 0;     // string escape / number / literal sub-state
  uint8_t key = 0;     // the open string is an object key
  uint8_t lit = 0;     // literal being matched (true / false / null)
  uint8_t depth = 0;   // open containers
  uint8_t ws = 0;      // current whitespace run
  uint8_t pad0 = 0, pad1 = 0;
  uint64_t stack = 0;  // bit i: container i is an object (else an array)
};

class JsonVocab {
 public:
  // tokens[i]: the bytes token i contributes to the decoded text ("" = never allowed, e.g. special
  // tokens); eos ids are allowed once the object is complete.
  JsonVocab(const std::vector<std::string>& tokens, const std::vector<int32_t>& eos_ids);
  int vocab_size() const { return (int)tokens_.size(); }
  int words() const { return (vocab_size() + 31) / 32; }
  const std::string& token(int id) const { return tokens_[id]; }
  bool is_eos(int id) const;
  size_t trie_nodes() const { return nodes_.size(); }
  size_t cache_entries() const;

  // allowed-token mask of state `s` under completion budget `limit` (bytes) -> out[words()];
  // returns the number of allowed tokens.  Cached per (state, limit).
  int mask(const JsonState& s, int limit, int max_depth, int max_ws, uint32_t* out);

  // Generic walk of the token trie from `node` in automaton state `s`: `step(state&, byte)` advances
  // a copy of the state (false = dead: the subtree is pruned), `leaf(state)` decides whether a
  // token ending in that state is allowed; allowed tokens are OR-ed into `out`.
  template <class S, class Step, class Leaf>
  void walk_tokens(int node, const S& s, Step& step, Leaf& leaf, uint32_t* out, int& count) const {
    for (int32_t ch = nodes_[node].child; ch >= 0; ch = nodes_[ch].sibling) {
      S t = s;
      if (!step(t, nodes_[ch].byte)) continue;
      if (nodes_[ch].tok >= 0 && leaf(t)) {
        for (int32_t k = nodes_[ch].tok; k >= 0; k = tok_next_[k]) {
          out[k >> 5] |= 1u << (k & 31);
          ++count;
        }
      }
      if (nodes_[ch].child >= 0) walk_tokens(ch, t, step, leaf, out, count);
    }
  }
  const std::vector<int32_t>& eos_ids() const { return eos_; }

 private:
  struct Node {
    int32_t child = -1, sibling = -1, tok = -1;  // tok: first token ending here (chain in tok_next_)
    uint8_t byte = 0;
  };
  std::vector<std::string> tokens_;
  std::vector<int32_t> eos_;
  std::vector<Node> nodes_;
  std::vector<int32_t> tok_next_;
  mutable std::mutex mu_;
  std::unordered_map<std::string, std::vector<uint32_t>> cache_;

  void walk(int node, const JsonState& s, int limit, int max_depth, int max_ws, uint32_t* out, int& count) const;
};

class JsonMatcher {
 public:
  JsonMatcher(std::shared_ptr<JsonVocab> vocab, int max_depth = 24, int max_ws = 8);
  // mask for the next token given `remaining` tokens in the budget (this one included); falls back
  // to the grammar alone if the budget leaves nothing, and to every token if even that is empty
  int fill_mask(int remaining, uint32_t* out);
  bool advance(int token);  // false: the token breaks the grammar (the matcher is then inert)
  bool done() const { return state_.mode == 11; }
  bool broken() const { return broken_; }
  int completion_len() const;
  std::string completion() const;
  const std::string& text() const { return text_; }

 private:
  std::shared_ptr<JsonVocab> vocab_;
  JsonState state_;
  int max_depth_, max_ws_;
  bool broken_ = false;
  std::string text_;
};

// JSON-Schema-constrained decoding: the schema is compiled (engine/json_schema.py) into a byte NFA
// (a regular language: fixed key order, typed / enumerated values, bounded whitespace), which is
// determinised lazily here; masks walk the token trie through the DFA and are cached per
// (DFA state, budget).  The budget rule is the JSON one: a token is allowed only if the shortest
// accepted completion after it fits in the tokens left.
class SchemaAutomaton {
 public:
  // edges: (from, lo, hi, to) byte-range transitions; eps: (from, to)
  SchemaAutomaton(std::shared_ptr<JsonVocab> vocab, int n_states, int start, const std::vector<int32_t>& accept,
                  const std::vector<std::vector<int32_t>>& edges, const std::vector<std::vector<int32_t>>& eps);
  int start() const { return start_; }
  int step(int d, uint8_t c);         // DFA transition (-1 = dead); builds states lazily
  // (intern() under mu_ in another thread's step / mask may reallocate acc_ / dist_ / sets_: read
  // them under the same lock -- automata are shared per tokenizer across engines and threads)
  bool accepting(int d) const {
    std::lock_guard<std::mutex> lk(mu_);
    return acc_[d] != 0;
  }
  int dist(int d) const {  // shortest accepted completion, bytes
    std::lock_guard<std::mutex> lk(mu_);
    return dist_[d];
  }
  bool has_exit(int d);               // any byte leads somewhere
  int mask(int d, int limit, uint32_t* out);
  int dfa_states() const {
    std::lock_guard<std::mutex> lk(mu_);
    return (int)sets_.size();
  }
  const JsonVocab& vocab() const { return *vocab_; }

 private:
  std::shared_ptr<JsonVocab> vocab_;
  int n_;
  std::vector<std::vector<std::pair<uint32_t, int32_t>>> tr_;  // per NFA state: (lo | hi << 8, to)
  std::vector<std::vector<int32_t>> eps_;
  std::vector<uint8_t> nacc_;
  std::vector<int32_t> ndist_;
  std::vector<std::vector<int32_t>> sets_;
  std::unordered_map<std::string, int32_t> ids_;
  std::vector<std::vector<int32_t>> trans_;  // [dfa][256]: -2 unknown, -1 dead
  std::vector<uint8_t> acc_;
  std::vector<int32_t> dist_;
  std::vector<int8_t> exit_;
  int start_;
  mutable std::mutex mu_;
  std::unordered_map<uint64_t, std::vector<uint32_t>> cache_;
  int intern(std::vector<int32_t> set);
  void closure(std::vector<int32_t>& set) const;
  int step_locked(int d, uint8_t c);
};

class SchemaMatcher {
 public:
  explicit SchemaMatcher(std::shared_ptr<SchemaAutomaton> a) : a_(std::move(a)), d_(a_->start()) {}
  int fill_mask(int remaining, uint32_t* out);
  bool advance(int token);
  bool done();
  bool broken() const { return broken_; }
  int completion_len() const { return a_->dist(d_); }
  const std::string& text() const { return text_; }

 private:
  std::shared_ptr<SchemaAutomaton> a_;
  int d_;
  bool broken_ = false;
  std::string text_;
};

// exposed for tests: feed raw bytes through the automaton
bool json_accepts(const std::string& bytes, bool require_complete, int max_depth = 64, int max_ws = 255);
int json_completion_len(const JsonState& s);
std::string json_completion(const JsonState& s);
bool json_step(JsonState& s, uint8_t c, int max_depth, int max_ws);

}  // namespace dab
