// JSON-constrained decoding (see json_grammar.h).
#include "runtime/json_grammar.h"

#include <algorithm>
#include <cstring>
#include <limits>

namespace dab {

namespace {

enum JsonMode : uint8_t {
  M_TOP = 0,     // before the top-level object
  M_OBJ_FIRST,   // after '{': key or '}'
  M_OBJ_KEY,     // after ',' in an object: key
  M_COLON,       // after a key
  M_VALUE,       // a value (after ':' or ',' in an array)
  M_ARR_FIRST,   // after '[': value or ']'
  M_OBJ_NEXT,    // after a member: ',' or '}'
  M_ARR_NEXT,    // after an element: ',' or ']'
  M_STR,         // inside a string (key or value)
  M_NUM,         // inside a number
  M_LIT,         // inside true / false / null
  M_DONE,        // the object is closed
};

// number sub-states; the "needs a digit" ones cannot end the number
enum NumSub : uint8_t { N_MINUS = 0, N_ZERO, N_INT, N_DOT, N_FRAC, N_E, N_ESIGN, N_EXP };

const char* const kLit[3] = {"true", "false", "null"};
const uint8_t kLitLen[3] = {4, 5, 4};

inline bool is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
inline bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
inline bool is_hex(uint8_t c) { return is_digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
inline bool top_is_obj(const JsonState& s) { return (s.stack >> (s.depth - 1)) & 1u; }

inline void after_value(JsonState& s) {
  s.ws = 0;
  if (s.depth == 0) s.mode = M_DONE;
  else s.mode = top_is_obj(s) ? M_OBJ_NEXT : M_ARR_NEXT;
}

inline bool push(JsonState& s, bool obj, int max_depth) {
  if (s.depth >= max_depth || s.depth >= 64) return false;
  if (obj) s.stack |= (uint64_t)1 << s.depth;
  else s.stack &= ~((uint64_t)1 << s.depth);
  ++s.depth;
  s.mode = obj ? M_OBJ_FIRST : M_ARR_FIRST;
  s.ws = 0;
  return true;
}

inline void pop(JsonState& s) {
  --s.depth;
  s.stack &= ((uint64_t)1 << s.depth) - 1;
  after_value(s);
}

inline bool take_ws(JsonState& s, uint8_t c, int max_ws) {
  if (!is_ws(c) || s.ws >= max_ws) return false;
  ++s.ws;
  return true;
}

bool begin_value(JsonState& s, uint8_t c, int max_depth) {
  s.ws = 0;
  switch (c) {
    case '{': return push(s, true, max_depth);
    case '[': return push(s, false, max_depth);
    case '"': s.mode = M_STR; s.key = 0; s.sub = 0; return true;
    case '-': s.mode = M_NUM; s.sub = N_MINUS; return true;
    case '0': s.mode = M_NUM; s.sub = N_ZERO; return true;
    case 't': s.mode = M_LIT; s.lit = 0; s.sub = 1; return true;
    case 'f': s.mode = M_LIT; s.lit = 1; s.sub = 1; return true;
    case 'n': s.mode = M_LIT; s.lit = 2; s.sub = 1; return true;
    default:
      if (c >= '1' && c <= '9') {
        s.mode = M_NUM;
        s.sub = N_INT;
        return true;
      }
      return false;
  }
}

}  // namespace

bool json_step(JsonState& s, uint8_t c, int max_depth, int max_ws) {
  switch (s.mode) {
    case M_TOP:
      if (c == '{') return push(s, true, max_depth);
      return take_ws(s, c, max_ws);
    case M_OBJ_FIRST:
    case M_OBJ_KEY:
      if (c == '"') {
        s.mode = M_STR;
        s.key = 1;
        s.sub = 0;
        s.ws = 0;
        return true;
      }
      if (c == '}' && s.mode == M_OBJ_FIRST) {
        pop(s);
        return true;
      }
      return take_ws(s, c, max_ws);
    case M_COLON:
      if (c == ':') {
        s.mode = M_VALUE;
        s.ws = 0;
        return true;
      }
      return take_ws(s, c, max_ws);
    case M_VALUE:
      if (is_ws(c)) return take_ws(s, c, max_ws);
      return begin_value(s, c, max_depth);
    case M_ARR_FIRST:
      if (c == ']') {
        pop(s);
        return true;
      }
      if (is_ws(c)) return take_ws(s, c, max_ws);
      return begin_value(s, c, max_depth);
    case M_OBJ_NEXT:
    case M_ARR_NEXT: {
      const bool obj = s.mode == M_OBJ_NEXT;
      if (c == ',') {
        s.mode = obj ? M_OBJ_KEY : M_VALUE;
        s.ws = 0;
        return true;
      }
      if (c == (obj ? '}' : ']')) {
        pop(s);
        return true;
      }
      return take_ws(s, c, max_ws);
    }
    case M_STR:
      if (s.sub == 0) {
        if (c == '"') {
          if (s.key) {
            s.key = 0;
            s.mode = M_COLON;
            s.ws = 0;
          } else {
            after_value(s);
          }
          return true;
        }
        if (c == '\\') {
          s.sub = 1;
          return true;
        }
        return c >= 0x20;
      }
      if (s.sub == 1) {
        if (c == 'u') {
          s.sub = 2;
          return true;
        }
        if (c == '"' || c == '\\' || c == '/' || c == 'b' || c == 'f' || c == 'n' || c == 'r' || c == 't') {
          s.sub = 0;
          return true;
        }
        return false;
      }
      if (!is_hex(c)) return false;  // \uXXXX: sub 2..5 count the hex digits
      s.sub = s.sub == 5 ? 0 : s.sub + 1;
      return true;
    case M_NUM:
      switch (s.sub) {
        case N_MINUS:
          if (c == '0') s.sub = N_ZERO;
          else if (c >= '1' && c <= '9') s.sub = N_INT;
          else return false;
          return true;
        case N_DOT:
          if (!is_digit(c)) return false;
          s.sub = N_FRAC;
          return true;
        case N_E:
          if (c == '+' || c == '-') s.sub = N_ESIGN;
          else if (is_digit(c)) s.sub = N_EXP;
          else return false;
          return true;
        case N_ESIGN:
          if (!is_digit(c)) return false;
          s.sub = N_EXP;
          return true;
        default:  // complete number: N_ZERO, N_INT, N_FRAC, N_EXP
          if (is_digit(c) && (s.sub == N_INT || s.sub == N_FRAC || s.sub == N_EXP)) return true;
          if (c == '.' && (s.sub == N_ZERO || s.sub == N_INT)) {
            s.sub = N_DOT;
            return true;
          }
          if ((c == 'e' || c == 'E') && s.sub != N_EXP) {
            s.sub = N_E;
            return true;
          }
          // the number ends here: the byte belongs to what follows it
          after_value(s);
          return json_step(s, c, max_depth, max_ws);
      }
    case M_LIT:
      if (c != (uint8_t)kLit[s.lit][s.sub]) return false;
      if (++s.sub == kLitLen[s.lit]) after_value(s);
      return true;
    case M_DONE:
      return take_ws(s, c, max_ws);
    default:
      return false;
  }
}

int json_completion_len(const JsonState& s) {
  const int d = s.depth;
  switch (s.mode) {
    case M_TOP: return 2;
    case M_OBJ_FIRST:
    case M_ARR_FIRST:
    case M_OBJ_NEXT:
    case M_ARR_NEXT: return d;
    case M_OBJ_KEY: return 4 + d;  // "":0
    case M_COLON: return 2 + d;    // :0
    case M_VALUE: return 1 + d;    // 0
    case M_STR: {
      int n = (s.key ? 3 : 1) + d;
      if (s.sub == 1) n += 1;
      else if (s.sub >= 2) n += 6 - s.sub;
      return n;
    }
    case M_NUM: {
      const bool need = s.sub == N_MINUS || s.sub == N_DOT || s.sub == N_E || s.sub == N_ESIGN;
      return (need ? 1 : 0) + d;
    }
    case M_LIT: return kLitLen[s.lit] - s.sub + d;
    default: return 0;
  }
}

std::string json_completion(const JsonState& s) {
  std::string out;
  switch (s.mode) {
    case M_TOP: return "{}";
    case M_OBJ_KEY: out = "\"\":0"; break;
    case M_COLON: out = ":0"; break;
    case M_VALUE: out = "0"; break;
    case M_STR:
      if (s.sub == 1) out = "n";
      else if (s.sub >= 2) out.assign(6 - s.sub, '0');
      out += s.key ? "\":0" : "\"";
      break;
    case M_NUM:
      if (s.sub == N_MINUS || s.sub == N_DOT || s.sub == N_E || s.sub == N_ESIGN) out = "0";
      break;
    case M_LIT: out = kLit[s.lit] + s.sub; break;
    default: break;
  }
  for (int i = s.depth - 1; i >= 0; --i) out.push_back(((s.stack >> i) & 1u) ? '}' : ']');
  return out;
}

bool json_accepts(const std::string& bytes, bool require_complete, int max_depth, int max_ws) {
  JsonState s;
  for (unsigned char c : bytes)
    if (!json_step(s, c, max_depth, max_ws)) return false;
  return !require_complete || s.mode == M_DONE;
}

// ---------------------------------------------------------------------------------------------
JsonVocab::JsonVocab(const std::vector<std::string>& tokens, const std::vector<int32_t>& eos_ids)
    : tokens_(tokens), eos_(eos_ids) {
  nodes_.emplace_back();  // root
  tok_next_.assign(tokens_.size(), -1);
  std::unordered_map<uint64_t, int32_t> edge;  // (node << 8 | byte) -> child
  edge.reserve(tokens_.size() * 4);
  for (size_t t = 0; t < tokens_.size(); ++t) {
    const std::string& b = tokens_[t];
    if (b.empty() || is_eos((int)t)) continue;
    int32_t n = 0;
    for (unsigned char c : b) {
      const uint64_t key = ((uint64_t)n << 8) | c;
      auto it = edge.find(key);
      if (it == edge.end()) {
        Node nd;
        nd.byte = c;
        nd.sibling = nodes_[n].child;
        const int32_t id = (int32_t)nodes_.size();
        nodes_.push_back(nd);
        nodes_[n].child = id;
        edge.emplace(key, id);
        n = id;
      } else {
        n = it->second;
      }
    }
    tok_next_[t] = nodes_[n].tok;
    nodes_[n].tok = (int32_t)t;
  }
}

bool JsonVocab::is_eos(int id) const { return std::find(eos_.begin(), eos_.end(), id) != eos_.end(); }

size_t JsonVocab::cache_entries() const {
  std::lock_guard<std::mutex> lk(mu_);
  return cache_.size();
}

void JsonVocab::walk(int node, const JsonState& s, int limit, int max_depth, int max_ws, uint32_t* out,
                     int& count) const {
  for (int32_t ch = nodes_[node].child; ch >= 0; ch = nodes_[ch].sibling) {
    JsonState t = s;
    if (!json_step(t, nodes_[ch].byte, max_depth, max_ws)) continue;
    if (nodes_[ch].tok >= 0 && json_completion_len(t) <= limit) {
      for (int32_t k = nodes_[ch].tok; k >= 0; k = tok_next_[k]) {
        out[k >> 5] |= 1u << (k & 31);
        ++count;
      }
    }
    if (nodes_[ch].child >= 0) walk(ch, t, limit, max_depth, max_ws, out, count);
  }
}

int JsonVocab::mask(const JsonState& s, int limit, int max_depth, int max_ws, uint32_t* out) {
  std::string key(reinterpret_cast<const char*>(&s), sizeof(JsonState));
  key.append(reinterpret_cast<const char*>(&limit), sizeof(int));
  key.append(reinterpret_cast<const char*>(&max_depth), sizeof(int));
  key.append(reinterpret_cast<const char*>(&max_ws), sizeof(int));
  const int W = words();
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = cache_.find(key);
    if (it != cache_.end()) {
      std::memcpy(out, it->second.data() + 1, W * sizeof(uint32_t));
      return (int)it->second[0];
    }
  }
  std::vector<uint32_t> m(W + 1, 0u);
  int count = 0;
  walk(0, s, limit, max_depth, max_ws, m.data() + 1, count);
  if (s.mode == M_DONE) {
    for (int32_t e : eos_)
      if (e >= 0 && e < vocab_size() && !(m[1 + (e >> 5)] & (1u << (e & 31)))) {
        m[1 + (e >> 5)] |= 1u << (e & 31);
        ++count;
      }
  }
  m[0] = (uint32_t)count;
  std::memcpy(out, m.data() + 1, W * sizeof(uint32_t));
  std::lock_guard<std::mutex> lk(mu_);
  if (cache_.size() >= 1024) cache_.clear();  // bounded: ~16 KB per entry at a 128k vocabulary
  cache_.emplace(std::move(key), std::move(m));
  return count;
}

// ---------------------------------------------------------------------------------------------
JsonMatcher::JsonMatcher(std::shared_ptr<JsonVocab> vocab, int max_depth, int max_ws)
    : vocab_(std::move(vocab)), max_depth_(std::max(1, std::min(max_depth, 64))), max_ws_(std::max(1, std::min(max_ws, 255))) {}

int JsonMatcher::fill_mask(int remaining, uint32_t* out) {
  const int W = vocab_->words();
  if (!broken_) {
    // tokens after this one: each can close at least one completion byte; a single token never
    // grows the completion by more than 64 bytes (keeps the unbounded mask one cache entry)
    const int slack = json_completion_len(state_) + 64;
    const int limit = std::min(std::max(remaining - 1, 0), slack);
    int n = vocab_->mask(state_, limit, max_depth_, max_ws_, out);
    if (n > 0) return n;
    n = vocab_->mask(state_, std::numeric_limits<int>::max() / 2, max_depth_, max_ws_, out);
    if (n > 0) return n;
  }
  std::fill(out, out + W, 0xFFFFFFFFu);
  const int V = vocab_->vocab_size();
  if (V % 32) out[W - 1] = (1u << (V % 32)) - 1;
  return V;
}

bool JsonMatcher::advance(int token) {
  if (broken_) return false;
  if (token < 0 || token >= vocab_->vocab_size()) {
    broken_ = true;
    return false;
  }
  if (vocab_->is_eos(token)) {
    if (state_.mode == M_DONE) return true;
    broken_ = true;
    return false;
  }
  JsonState s = state_;
  const std::string& b = vocab_->token(token);
  if (b.empty()) {
    broken_ = true;
    return false;
  }
  for (unsigned char c : b) {
    if (!json_step(s, c, max_depth_, max_ws_)) {
      broken_ = true;
      return false;
    }
  }
  state_ = s;
  text_ += b;
  return true;
}

int JsonMatcher::completion_len() const { return json_completion_len(state_); }

std::string JsonMatcher::completion() const { return json_completion(state_); }

}  // namespace dab
