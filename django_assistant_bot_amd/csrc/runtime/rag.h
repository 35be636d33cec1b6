// Host-side retrieval post-processing (native).
//
// aggregate_documents() is the exact semantics of the reference's broad document search
// (rag/services/search_service.py:133-152): hits arrive sorted by ascending cosine distance,
// they are grouped by document id preserving that order, documents with fewer than
// `max_scores_n` hits are dropped, a document scores 1 - mean(first max_scores_n distances),
// and the best `top_n` documents are returned (ties broken by ascending document id).
#pragma once
#include <cstdint>
#include <vector>

namespace dab {

struct DocScore {
  int64_t doc_id;
  double score;
};

std::vector<DocScore> aggregate_documents(const float* distances, const int64_t* doc_ids, int n_hits,
                                          int max_scores_n, int top_n);

// Merges S sorted-descending partial top-k lists (similarities, ids) into the global top-k.
void merge_topk(const float* vals, const int64_t* ids, int S, int k_in, int k_out, float* out_vals,
                int64_t* out_ids);

}  // namespace dab
