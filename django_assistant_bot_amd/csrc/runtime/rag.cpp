#include "rag.h"

#include <algorithm>
#include <cmath>
#include <queue>
#include <unordered_map>

namespace dab {

std::vector<DocScore> aggregate_documents(const float* distances, const int64_t* doc_ids, int n_hits,
                                          int max_scores_n, int top_n) {
  std::vector<DocScore> out;
  if (max_scores_n <= 0 || top_n <= 0) return out;
  struct Acc {
    int count = 0;
    double sum = 0.0;
  };
  std::unordered_map<int64_t, Acc> acc;
  acc.reserve((size_t)n_hits);
  for (int i = 0; i < n_hits; ++i) {
    if (!std::isfinite(distances[i])) continue;  // filtered-out rows never count as hits
    Acc& a = acc[doc_ids[i]];
    if (a.count < max_scores_n) a.sum += distances[i];
    ++a.count;
  }
  for (auto& kv : acc) {
    if (kv.second.count >= max_scores_n) out.push_back({kv.first, 1.0 - kv.second.sum / max_scores_n});
  }
  std::sort(out.begin(), out.end(), [](const DocScore& a, const DocScore& b) {
    if (a.score != b.score) return a.score > b.score;
    return a.doc_id < b.doc_id;
  });
  if ((int)out.size() > top_n) out.resize(top_n);
  return out;
}

void merge_topk(const float* vals, const int64_t* ids, int S, int k_in, int k_out, float* out_vals,
                int64_t* out_ids) {
  // k-way merge of descending lists with a max-heap of list heads
  typedef std::pair<float, std::pair<int64_t, int>> Item;  // (value, (-id, list))
  auto cmp = [](const Item& a, const Item& b) {
    if (a.first != b.first) return a.first < b.first;
    return a.second.first < b.second.first;
  };
  std::priority_queue<Item, std::vector<Item>, decltype(cmp)> heap(cmp);
  std::vector<int> pos(S, 0);
  for (int s = 0; s < S; ++s)
    if (k_in > 0) heap.push({vals[(size_t)s * k_in], {-ids[(size_t)s * k_in], s}});
  int n = 0;
  while (n < k_out && !heap.empty()) {
    Item it = heap.top();
    heap.pop();
    const int s = it.second.second;
    out_vals[n] = it.first;
    out_ids[n] = -it.second.first;
    ++n;
    if (++pos[s] < k_in) heap.push({vals[(size_t)s * k_in + pos[s]], {-ids[(size_t)s * k_in + pos[s]], s}});
  }
  for (; n < k_out; ++n) {
    out_vals[n] = -INFINITY;
    out_ids[n] = -1;
  }
}

}  // namespace dab
