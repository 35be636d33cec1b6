"""Per-document score aggregation of question/sentence hits (reference rag/services/search_service.py:
133-152), Django-free.  Hits arrive sorted by ascending cosine distance; documents with fewer than
``max_scores_n`` hits are dropped; score = 1 - mean(first max_scores_n distances).  Uses the native
implementation (csrc/runtime/rag.cpp) when the extension is present."""
from __future__ import annotations

from collections import OrderedDict


def aggregate_documents(distances, doc_ids, max_scores_n: int, top_n: int) -> list:
    """-> [(doc_id, score)] best first, at most ``top_n``; ties by ascending doc id."""
    try:
        import numpy as np

        from django_assistant_bot_amd.ops import native

        return [(int(d), float(s)) for d, s in native().aggregate_documents(
            np.asarray(distances, dtype=np.float32), np.asarray(doc_ids, dtype=np.int64), max_scores_n, top_n)]
    except Exception:
        pass
    groups: "OrderedDict[int, list]" = OrderedDict()
    for d, doc in zip(distances, doc_ids):
        if d == float("inf") or d != d:
            continue
        groups.setdefault(int(doc), []).append(float(d))
    scored = [(doc, 1.0 - sum(v[:max_scores_n]) / max_scores_n) for doc, v in groups.items() if len(v) >= max_scores_n]
    scored.sort(key=lambda x: (-x[1], x[0]))
    return scored[:top_n]
