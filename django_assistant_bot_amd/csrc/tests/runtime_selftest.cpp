// Host-only self test of the native runtime (no HIP): randomized KV block manager traffic with
// invariant checks, multi-threaded tokenizer batch encode vs sequential encode, document
// aggregation and top-k merge vs brute force.  Built by `python -m django_assistant_bot_amd.build
// --selftest asan|tsan` with -fsanitize=address,undefined (or thread) so the sanitizers watch the
// same code the extension links (sanitizers on host code).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <numeric>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "runtime/kv_manager.h"
#include "runtime/rag.h"
#include "runtime/tokenizer.h"
#include "runtime/trace.h"

static int failures = 0;
#define CHECK(cond, ...)                                       \
  do {                                                         \
    if (!(cond)) {                                             \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                       \
      std::fprintf(stderr, "\n");                              \
      ++failures;                                              \
    }                                                          \
  } while (0)

static void test_kv_manager(unsigned seed) {
  const int NB = 96, BS = 16, MAXB = 32;
  dab::KVBlockManager m(NB, BS, true);
  std::mt19937 rng(seed);
  std::map<int64_t, int> live;  // seq -> tokens
  int64_t next_id = 0;
  std::vector<int32_t> shared_prefix(40);
  std::iota(shared_prefix.begin(), shared_prefix.end(), 7);
  for (int it = 0; it < 4000; ++it) {
    const int op = rng() % 10;
    if (op < 4) {  // admit, half of them sharing a cached prefix
      std::vector<int32_t> toks = (rng() & 1) ? shared_prefix : std::vector<int32_t>();
      const int extra = 1 + rng() % 60;
      for (int i = 0; i < extra; ++i) toks.push_back((int32_t)(rng() % 5000));
      const int64_t id = next_id++;
      const int cached = m.add_sequence(id, toks, 1);
      if (cached < 0) continue;
      CHECK(cached <= (int)toks.size() - 1, "cached %d of %zu", cached, toks.size());
      CHECK(cached % BS == 0, "cached prefix not block aligned: %d", cached);
      m.commit_prefix(id, (int)toks.size());
      live[id] = (int)toks.size();
      std::vector<int64_t> slots(toks.size());
      m.slot_mapping(id, 0, (int)toks.size(), slots.data());
      for (int64_t s : slots) CHECK(s >= 0 && s < (int64_t)NB * BS, "slot %lld out of range", (long long)s);
    } else if (op < 8 && !live.empty()) {  // decode step over every live sequence
      std::vector<int64_t> ids;
      std::vector<int32_t> last;
      for (auto& kv : live) {
        ids.push_back(kv.first);
        last.push_back((int32_t)(rng() % 5000));
      }
      const size_t B = ids.size();
      std::vector<int32_t> tid(B), pos(B), ctx(B), bt(B * MAXB);
      std::vector<int64_t> slots(B);
      const int fail = m.prepare_decode(ids, last, MAXB, tid.data(), pos.data(), slots.data(), ctx.data(), bt.data());
      if (fail >= 0) {  // preempt the failing sequence like the engine does
        m.free_sequence(ids[fail]);
        live.erase(ids[fail]);
        continue;
      }
      std::set<int64_t> uniq(slots.begin(), slots.end());
      CHECK(uniq.size() == B, "decode slots collide");
      for (size_t b = 0; b < B; ++b) {
        CHECK(pos[b] == live[ids[b]], "position %d != length %d", pos[b], live[ids[b]]);
        CHECK(ctx[b] == pos[b] + 1, "ctx");
        CHECK(slots[b] / BS == bt[b * MAXB + pos[b] / BS], "slot not in the block table");
        live[ids[b]] += 1;
      }
    } else if (!live.empty()) {  // finish one
      auto itr = live.begin();
      std::advance(itr, rng() % live.size());
      m.free_sequence(itr->first);
      live.erase(itr);
    }
    // no block is owned by two live sequences unless it is a shared (cached) prefix block
    std::map<int32_t, int> owners;
    for (auto& kv : live)
      for (int32_t b : m.blocks(kv.first)) owners[b]++;
    int used = (int)owners.size();
    CHECK(used + m.num_free_blocks() <= NB, "blocks leaked or double counted: used %d free %d", used,
          m.num_free_blocks());
    for (auto& kv : live) CHECK(m.capacity_tokens(kv.first) >= kv.second, "capacity < tokens");
  }
  for (auto& kv : live) m.free_sequence(kv.first);
  CHECK(m.num_free_blocks() == NB, "blocks not returned: %d of %d", m.num_free_blocks(), NB);
}

static void test_tokenizer() {
  dab::TokenizerConfig cfg;
  dab::HashTokenizer tok(cfg);
  std::vector<std::string> texts;
  std::mt19937 rng(3);
  const char* words[] = {"account", "billing", "Привет", "мир", "über", "naïve", "x", "supercalifragilisticexpialidocious",
                         "42", "?", "hello,", "world."};
  for (int i = 0; i < 500; ++i) {
    std::string t;
    for (int j = 0, n = 1 + rng() % 40; j < n; ++j) t += std::string(words[rng() % 12]) + " ";
    texts.push_back(t);
  }
  std::vector<int32_t> flat;
  std::vector<int64_t> offs;
  tok.encode_batch(texts, true, 64, 8, flat, offs);
  CHECK(offs.size() == texts.size() + 1, "offsets");
  for (size_t i = 0; i < texts.size(); ++i) {
    auto one = tok.encode(texts[i], true, 64);
    std::vector<int32_t> got(flat.begin() + offs[i], flat.begin() + offs[i + 1]);
    CHECK(one == got, "batch encode differs from encode at %zu", i);
    CHECK(!got.empty() && got.front() == cfg.cls_id && got.back() == cfg.sep_id, "framing");
  }
  auto ids = tok.encode_raw("account billing", true);
  CHECK(tok.decode(ids, true) == "account billing", "decode round trip: '%s'", tok.decode(ids, true).c_str());
}

static void test_rag() {
  std::mt19937 rng(5);
  for (int trial = 0; trial < 200; ++trial) {
    const int n = 1 + rng() % 250, m = 1 + rng() % 5, top = 1 + rng() % 5;
    std::vector<float> d(n);
    std::vector<int64_t> doc(n);
    for (int i = 0; i < n; ++i) {
      d[i] = (float)(rng() % 1000) / 1000.f;
      doc[i] = rng() % 40;
    }
    std::vector<int> order(n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return d[a] < d[b]; });
    std::vector<float> ds(n);
    std::vector<int64_t> docs(n);
    for (int i = 0; i < n; ++i) {
      ds[i] = d[order[i]];
      docs[i] = doc[order[i]];
    }
    auto got = dab::aggregate_documents(ds.data(), docs.data(), n, m, top);
    // brute force
    std::map<int64_t, std::vector<float>> by;
    for (int i = 0; i < n; ++i) by[docs[i]].push_back(ds[i]);
    std::vector<std::pair<double, int64_t>> exp;
    for (auto& kv : by) {
      if ((int)kv.second.size() < m) continue;
      double s = 0;
      for (int i = 0; i < m; ++i) s += kv.second[i];
      exp.push_back({1.0 - s / m, kv.first});
    }
    std::sort(exp.begin(), exp.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first > b.first : a.second < b.second; });
    if ((int)exp.size() > top) exp.resize(top);
    CHECK(got.size() == exp.size(), "aggregate size %zu vs %zu", got.size(), exp.size());
    for (size_t i = 0; i < std::min(got.size(), exp.size()); ++i)
      CHECK(got[i].doc_id == exp[i].second && std::abs(got[i].score - exp[i].first) < 1e-6, "aggregate mismatch");
  }
  // top-k merge of S sorted lists
  const int S = 4, K = 50;
  std::vector<float> vals(S * K);
  std::vector<int64_t> ids(S * K);
  for (int s = 0; s < S; ++s) {
    for (int k = 0; k < K; ++k) {
      vals[s * K + k] = (float)(rng() % 100000) / 100000.f;
      ids[s * K + k] = s * 1000 + k;
    }
    std::sort(vals.begin() + s * K, vals.begin() + (s + 1) * K, std::greater<float>());
  }
  std::vector<float> ov(K);
  std::vector<int64_t> oi(K);
  dab::merge_topk(vals.data(), ids.data(), S, K, K, ov.data(), oi.data());
  std::vector<float> all(vals);
  std::sort(all.begin(), all.end(), std::greater<float>());
  for (int k = 0; k < K; ++k) CHECK(ov[k] == all[k], "merge_topk value %d", k);
}

int main() {
  for (unsigned seed = 1; seed <= 4; ++seed) test_kv_manager(seed);
  test_tokenizer();
  test_rag();
  dab::trace::range_push("selftest");  // no-op or real: must not crash either way
  dab::trace::range_pop();
  if (failures) {
    std::fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  std::printf("runtime selftest ok\n");
  return 0;
}
