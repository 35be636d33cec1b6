// JSON-constrained decoding (see json_grammar.h).
#include "runtime/json_grammar.h"

#include <algorithm>
#include <cstring>
#include <deque>
#include <limits>
#include <stdexcept>

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
    case '"': s.mode = M_STR; s.key = 0; s.sub = 0; s.lit = 0; return true;
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
        s.lit = 0;
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
        // UTF-8 structure inside strings (byte-level tokens can split characters): `lit` counts
        // the continuation bytes still owed by the last lead byte
        if (s.lit) {
          if (c < 0x80 || c > 0xBF) return false;
          --s.lit;
          return true;
        }
        if (c >= 0x80) {
          if (c >= 0xC2 && c <= 0xDF) s.lit = 1;
          else if (c >= 0xE0 && c <= 0xEF) s.lit = 2;
          else if (c >= 0xF0 && c <= 0xF4) s.lit = 3;
          else return false;
          return true;
        }
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
      int n = (s.key ? 3 : 1) + d + s.lit;
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
      out.assign(s.lit, '\x80');
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

// ---------------------------------------------------------------------------------------------
SchemaAutomaton::SchemaAutomaton(std::shared_ptr<JsonVocab> vocab, int n_states, int start,
                                 const std::vector<int32_t>& accept, const std::vector<std::vector<int32_t>>& edges,
                                 const std::vector<std::vector<int32_t>>& eps)
    : vocab_(std::move(vocab)), n_(n_states), tr_(n_states), eps_(n_states), nacc_(n_states, 0) {
  for (const auto& e : edges) {
    if (e.size() != 4 || e[0] < 0 || e[0] >= n_ || e[3] < 0 || e[3] >= n_ || e[1] < 0 || e[2] > 255 || e[1] > e[2])
      throw std::invalid_argument("schema NFA: bad edge");
    tr_[e[0]].emplace_back((uint32_t)e[1] | ((uint32_t)e[2] << 8), e[3]);
  }
  std::vector<std::vector<int32_t>> reps(n_);  // reverse epsilon edges
  std::vector<std::vector<int32_t>> rtr(n_);   // reverse byte edges
  for (const auto& e : eps) {
    if (e.size() != 2 || e[0] < 0 || e[0] >= n_ || e[1] < 0 || e[1] >= n_)
      throw std::invalid_argument("schema NFA: bad epsilon edge");
    eps_[e[0]].push_back(e[1]);
    reps[e[1]].push_back(e[0]);
  }
  for (int u = 0; u < n_; ++u)
    for (const auto& t : tr_[u]) rtr[t.second].push_back(u);
  // shortest accepted completion of every NFA state: 0-1 BFS backwards from the accept states
  ndist_.assign(n_, std::numeric_limits<int32_t>::max() / 4);
  std::deque<int32_t> q;
  for (int32_t a : accept) {
    if (a < 0 || a >= n_) throw std::invalid_argument("schema NFA: bad accept state");
    nacc_[a] = 1;
    ndist_[a] = 0;
    q.push_back(a);
  }
  while (!q.empty()) {
    const int32_t v = q.front();
    q.pop_front();
    for (int32_t u : reps[v])
      if (ndist_[v] < ndist_[u]) {
        ndist_[u] = ndist_[v];
        q.push_front(u);
      }
    for (int32_t u : rtr[v])
      if (ndist_[v] + 1 < ndist_[u]) {
        ndist_[u] = ndist_[v] + 1;
        q.push_back(u);
      }
  }
  if (start < 0 || start >= n_) throw std::invalid_argument("schema NFA: bad start state");
  start_ = intern({start});
}

void SchemaAutomaton::closure(std::vector<int32_t>& set) const {
  std::vector<uint8_t> seen(n_, 0);
  std::vector<int32_t> stack(set.begin(), set.end());
  set.clear();
  while (!stack.empty()) {
    const int32_t u = stack.back();
    stack.pop_back();
    if (seen[u]) continue;
    seen[u] = 1;
    set.push_back(u);
    for (int32_t v : eps_[u])
      if (!seen[v]) stack.push_back(v);
  }
  std::sort(set.begin(), set.end());
}

int SchemaAutomaton::intern(std::vector<int32_t> set) {
  closure(set);
  std::string key(reinterpret_cast<const char*>(set.data()), set.size() * sizeof(int32_t));
  auto it = ids_.find(key);
  if (it != ids_.end()) return it->second;
  const int32_t id = (int32_t)sets_.size();
  uint8_t acc = 0;
  int32_t dist = std::numeric_limits<int32_t>::max() / 4;
  for (int32_t u : set) {
    acc |= nacc_[u];
    dist = std::min(dist, ndist_[u]);
  }
  sets_.push_back(std::move(set));
  ids_.emplace(std::move(key), id);
  trans_.emplace_back(256, -2);
  acc_.push_back(acc);
  dist_.push_back(dist);
  exit_.push_back(-1);
  return id;
}

int SchemaAutomaton::step_locked(int d, uint8_t c) {
  int32_t& t = trans_[d][c];
  if (t != -2) return t;
  std::vector<int32_t> next;
  for (int32_t u : sets_[d])
    for (const auto& e : tr_[u])
      if (c >= (e.first & 255u) && c <= (e.first >> 8)) next.push_back(e.second);
  const int32_t r = next.empty() ? -1 : intern(std::move(next));
  trans_[d][c] = r;  // intern may have grown trans_: index again
  return r;
}

int SchemaAutomaton::step(int d, uint8_t c) {
  std::lock_guard<std::mutex> lk(mu_);
  return step_locked(d, c);
}

bool SchemaAutomaton::has_exit(int d) {
  std::lock_guard<std::mutex> lk(mu_);
  if (exit_[d] < 0) {
    int8_t any = 0;
    for (int c = 0; c < 256 && !any; ++c) any = step_locked(d, (uint8_t)c) >= 0;
    exit_[d] = any;
  }
  return exit_[d] != 0;
}

int SchemaAutomaton::mask(int d, int limit, uint32_t* out) {
  const int W = vocab_->words();
  const uint64_t key = ((uint64_t)(uint32_t)d << 32) | (uint32_t)limit;
  std::lock_guard<std::mutex> lk(mu_);
  auto it = cache_.find(key);
  if (it != cache_.end()) {
    std::memcpy(out, it->second.data() + 1, W * sizeof(uint32_t));
    return (int)it->second[0];
  }
  std::vector<uint32_t> m(W + 1, 0u);
  int count = 0;
  auto step = [this](int& s, uint8_t c) {
    s = step_locked(s, c);
    return s >= 0;
  };
  auto leaf = [this, limit](int s) { return dist_[s] <= limit; };
  vocab_->walk_tokens(0, d, step, leaf, m.data() + 1, count);
  if (acc_[d]) {
    for (int32_t e : vocab_->eos_ids())
      if (e >= 0 && e < vocab_->vocab_size() && !(m[1 + (e >> 5)] & (1u << (e & 31)))) {
        m[1 + (e >> 5)] |= 1u << (e & 31);
        ++count;
      }
  }
  m[0] = (uint32_t)count;
  std::memcpy(out, m.data() + 1, W * sizeof(uint32_t));
  if (cache_.size() >= 256) cache_.clear();  // per schema: <= 4 MB at a 128k vocabulary
  cache_.emplace(key, std::move(m));
  return count;
}

int SchemaMatcher::fill_mask(int remaining, uint32_t* out) {
  const JsonVocab& v = a_->vocab();
  const int W = v.words();
  if (!broken_) {
    const int slack = a_->dist(d_) + 64;
    int n = a_->mask(d_, std::min(std::max(remaining - 1, 0), slack), out);
    if (n > 0) return n;
    n = a_->mask(d_, std::numeric_limits<int>::max() / 8, out);
    if (n > 0) return n;
  }
  std::fill(out, out + W, 0xFFFFFFFFu);
  const int V = v.vocab_size();
  if (V % 32) out[W - 1] = (1u << (V % 32)) - 1;
  return V;
}

bool SchemaMatcher::advance(int token) {
  const JsonVocab& v = a_->vocab();
  if (broken_) return false;
  if (token < 0 || token >= v.vocab_size()) {
    broken_ = true;
    return false;
  }
  if (v.is_eos(token)) {
    if (a_->accepting(d_)) return true;
    broken_ = true;
    return false;
  }
  const std::string& b = v.token(token);
  int d = d_;
  for (unsigned char c : b) {
    d = a_->step(d, c);
    if (d < 0) break;
  }
  if (b.empty() || d < 0) {
    broken_ = true;
    return false;
  }
  d_ = d;
  text_ += b;
  return true;
}

bool SchemaMatcher::done() { return !broken_ && a_->accepting(d_) && !a_->has_exit(d_); }

}  // namespace dab
