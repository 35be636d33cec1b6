#include "tokenizer.h"

#include <algorithm>
#include <cstdint>
#include <thread>

namespace dab {

namespace {

// Decodes one UTF-8 code point starting at s[i]; advances i.  Invalid bytes map to U+FFFD.
uint32_t next_cp(const std::string& s, size_t& i) {
  const unsigned char c = (unsigned char)s[i];
  if (c < 0x80) {
    i += 1;
    return c;
  }
  int n = 0;
  uint32_t cp = 0;
  if ((c & 0xE0) == 0xC0) {
    n = 1;
    cp = c & 0x1F;
  } else if ((c & 0xF0) == 0xE0) {
    n = 2;
    cp = c & 0x0F;
  } else if ((c & 0xF8) == 0xF0) {
    n = 3;
    cp = c & 0x07;
  } else {
    i += 1;
    return 0xFFFD;
  }
  for (int k = 1; k <= n; ++k) {
    if (i + k >= s.size()) {
      i = s.size();
      return 0xFFFD;
    }
    const unsigned char cc = (unsigned char)s[i + k];
    if ((cc & 0xC0) != 0x80) {
      i += k;
      return 0xFFFD;
    }
    cp = (cp << 6) | (cc & 0x3F);
  }
  i += n + 1;
  return cp;
}

void put_cp(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out.push_back((char)cp);
  } else if (cp < 0x800) {
    out.push_back((char)(0xC0 | (cp >> 6)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    out.push_back((char)(0xE0 | (cp >> 12)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    out.push_back((char)(0xF0 | (cp >> 18)));
    out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

bool is_space(uint32_t cp) { return cp == ' ' || cp == '\t' || cp == '\n' || cp == '\r' || cp == 0xA0 || cp == 0x3000; }

bool is_word_char(uint32_t cp) {
  if ((cp >= '0' && cp <= '9') || (cp >= 'a' && cp <= 'z') || (cp >= 'A' && cp <= 'Z') || cp == '_') return true;
  if (cp >= 0xC0 && cp <= 0x24F && cp != 0xD7 && cp != 0xF7) return true;  // Latin-1 / extended letters
  if (cp >= 0x400 && cp <= 0x4FF) return true;                                  // Cyrillic
  if (cp >= 0x370 && cp <= 0x3FF) return true;                                  // Greek
  if (cp >= 0x4E00 && cp <= 0x9FFF) return false;  // CJK: one token per ideograph
  if (cp >= 0x3040 && cp <= 0x30FF) return false;  // kana
  return cp >= 0x80 && cp != 0xFFFD && !(cp >= 0x2000 && cp <= 0x2BFF);
}

uint32_t lower(uint32_t cp) {
  if (cp >= 'A' && cp <= 'Z') return cp + 32;
  if (cp >= 0x410 && cp <= 0x42F) return cp + 32;   // А-Я
  if (cp >= 0x400 && cp <= 0x40F) return cp + 80;   // Ѐ-Џ
  if (cp >= 0xC0 && cp <= 0xDE && cp != 0xD7) return cp + 32;
  return cp;
}

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

template <class F>
void split_words(const std::string& text, int max_chars, F emit) {
  std::string cur;
  int cur_chars = 0;
  size_t i = 0;
  auto flush = [&]() {
    if (!cur.empty()) emit(cur);
    cur.clear();
    cur_chars = 0;
  };
  while (i < text.size()) {
    const uint32_t cp = lower(next_cp(text, i));
    if (is_space(cp)) {
      flush();
    } else if (is_word_char(cp)) {
      put_cp(cur, cp);
      if (++cur_chars >= max_chars) flush();
    } else {
      flush();
      std::string p;
      put_cp(p, cp);
      emit(p);
    }
  }
  flush();
}

}  // namespace

int32_t HashTokenizer::word_id(const std::string& w) const {
  const uint64_t span = (uint64_t)std::max(1, cfg_.last_id - cfg_.first_id);
  return (int32_t)(cfg_.first_id + (int64_t)(fnv1a(w) % span));
}

std::vector<int32_t> HashTokenizer::encode_raw(const std::string& text, bool remember) const {
  std::vector<int32_t> out;
  out.reserve(text.size() / 4 + 4);
  std::vector<std::pair<int32_t, std::string>> fresh;
  split_words(text, cfg_.max_word_chars, [&](const std::string& w) {
    const int32_t id = word_id(w);
    out.push_back(id);
    if (remember) fresh.emplace_back(id, w);
  });
  if (remember && !fresh.empty()) {
    std::lock_guard<std::mutex> lk(mu_);
    if (seen_.size() < (size_t)4000000) {
      for (auto& kv : fresh) seen_.emplace(kv.first, kv.second);
    }
  }
  return out;
}

std::vector<int32_t> HashTokenizer::encode(const std::string& text, bool add_special, int max_len) const {
  std::vector<int32_t> raw = encode_raw(text, true);
  std::vector<int32_t> out;
  const bool has_cls = add_special && cfg_.cls_id >= 0;
  const bool has_sep = add_special && cfg_.sep_id >= 0;
  const int extra = (int)has_cls + (int)has_sep;
  size_t keep = raw.size();
  if (max_len > 0 && (int)keep + extra > max_len) keep = (size_t)std::max(0, max_len - extra);
  out.reserve(keep + extra);
  if (has_cls) out.push_back(cfg_.cls_id);
  out.insert(out.end(), raw.begin(), raw.begin() + keep);
  if (has_sep) out.push_back(cfg_.sep_id);
  return out;
}

void HashTokenizer::encode_into(const std::string& text, bool add_special, int max_len, std::vector<int32_t>& out,
                                std::vector<uint8_t>& mark,
                                std::vector<std::pair<int32_t, std::string>>& fresh) const {
  const bool has_cls = add_special && cfg_.cls_id >= 0;
  const bool has_sep = add_special && cfg_.sep_id >= 0;
  const size_t extra = (size_t)has_cls + (size_t)has_sep;
  const size_t cap = max_len > 0 ? (size_t)std::max<int>(0, max_len - (int)extra) : SIZE_MAX;
  out.clear();
  if (has_cls) out.push_back(cfg_.cls_id);
  size_t kept = 0;
  split_words(text, cfg_.max_word_chars, [&](const std::string& w) {
    if (kept >= cap) return;
    const int32_t id = word_id(w);
    out.push_back(id);
    ++kept;
    if ((size_t)id < mark.size() && !mark[id]) {
      mark[id] = 1;
      fresh.emplace_back(id, w);
    }
  });
  if (has_sep) out.push_back(cfg_.sep_id);
}

void HashTokenizer::remember(std::vector<std::pair<int32_t, std::string>>& fresh) const {
  if (fresh.empty()) return;
  std::lock_guard<std::mutex> lk(mu_);
  if (seen_.size() >= (size_t)4000000) return;
  for (auto& kv : fresh) seen_.emplace(kv.first, std::move(kv.second));
}

// Each worker encodes a contiguous range of texts with its own first-seen marks (one byte per id),
// so the decode table is updated once per worker with the distinct words it met, instead of one
// locked map insert per text (which serialised the workers: 8 threads ran at 1.25x one thread).
void HashTokenizer::encode_batch(const std::vector<std::string>& texts, bool add_special, int max_len, int threads,
                                 std::vector<int32_t>& ids, std::vector<int64_t>& offsets) const {
  const size_t n = texts.size();
  threads = std::max(1, std::min<int>(threads, (int)std::max<size_t>(1, n / 64)));
  std::vector<std::vector<int32_t>> chunk_ids(threads);
  std::vector<std::vector<int64_t>> chunk_lens(threads);
  std::vector<std::thread> pool;
  const size_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    pool.emplace_back([&, t]() {
      const size_t lo = std::min(n, t * per), hi = std::min(n, lo + per);
      std::vector<uint8_t> mark((size_t)std::max(cfg_.vocab_size, cfg_.last_id), 0);
      std::vector<std::pair<int32_t, std::string>> fresh;
      std::vector<int32_t> one;
      auto& dst = chunk_ids[t];
      auto& lens = chunk_lens[t];
      lens.reserve(hi - lo);
      for (size_t i = lo; i < hi; ++i) {
        encode_into(texts[i], add_special, max_len, one, mark, fresh);
        dst.insert(dst.end(), one.begin(), one.end());
        lens.push_back((int64_t)one.size());
      }
      remember(fresh);
    });
  }
  for (auto& th : pool) th.join();
  offsets.assign(n + 1, 0);
  size_t i = 0;
  for (int t = 0; t < threads; ++t)
    for (int64_t len : chunk_lens[t]) {
      offsets[i + 1] = offsets[i] + len;
      ++i;
    }
  ids.resize(offsets[n]);
  size_t pos = 0;
  for (int t = 0; t < threads; ++t) {
    std::copy(chunk_ids[t].begin(), chunk_ids[t].end(), ids.begin() + pos);
    pos += chunk_ids[t].size();
  }
}

std::string HashTokenizer::pseudo_word(int32_t id) const {
  static const char* syl[] = {"ka", "lo", "mi", "ne", "ru", "sa", "ti", "vo", "ze", "da",
                              "pe", "qu", "ri", "so", "tu", "va", "we", "xi", "yo", "bu"};
  std::string w;
  uint32_t x = (uint32_t)id * 2654435761u;
  const int n = 1 + (int)(x % 3);
  for (int k = 0; k < n; ++k) {
    w += syl[x % 20];
    x /= 20;
    x += (uint32_t)id;
  }
  return w;
}

std::string HashTokenizer::decode(const std::vector<int32_t>& ids, bool skip_special) const {
  std::string out;
  std::lock_guard<std::mutex> lk(mu_);
  for (int32_t id : ids) {
    const bool special = id == cfg_.pad_id || id == cfg_.cls_id || id == cfg_.sep_id || id == cfg_.unk_id ||
                         id < cfg_.first_id || id >= cfg_.last_id;
    if (special && skip_special) continue;
    std::string w;
    auto it = seen_.find(id);
    if (it != seen_.end()) w = it->second;
    else if (special) w = "[" + std::to_string(id) + "]";
    else w = pseudo_word(id);
    const bool punct = w.size() == 1 && !((w[0] >= 'a' && w[0] <= 'z') || (w[0] >= '0' && w[0] <= '9'));
    if (!out.empty() && !punct) out.push_back(' ');
    out += w;
  }
  return out;
}

std::vector<std::string> HashTokenizer::token_texts() const {
  std::vector<std::string> out(cfg_.vocab_size);
  std::lock_guard<std::mutex> lk(mu_);
  for (int32_t id = 0; id < cfg_.vocab_size; ++id) {
    const bool special = id == cfg_.pad_id || id == cfg_.cls_id || id == cfg_.sep_id || id == cfg_.unk_id ||
                         id < cfg_.first_id || id >= cfg_.last_id;
    if (special) continue;
    auto it = seen_.find(id);
    const std::string w = it != seen_.end() ? it->second : pseudo_word(id);
    const bool punct = w.size() == 1 && !((w[0] >= 'a' && w[0] <= 'z') || (w[0] >= '0' && w[0] <= '9'));
    out[id] = punct ? w : " " + w;
  }
  return out;
}

int64_t HashTokenizer::count_words(const std::string& text) {
  int64_t n = 0;
  bool in = false;
  for (unsigned char c : text) {
    const bool sp = c == ' ' || c == '\t' || c == '\n' || c == '\r';
    if (!sp && !in) ++n;
    in = !sp;
  }
  return n;
}

}  // namespace dab
