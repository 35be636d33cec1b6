"""Embedding search over the knowledge base (reference rag/services/search_service.py:17-196).

Public API unchanged: ``cosine_similarity``, ``embeddings_similarity``, ``get_embedding``,
``embedding_search(query, qs, max_scores_n=10, top_n=10)``, ``embedding_search_{documents,questions,
sentences}(query_embedding, qs, n)`` and ``_objects_embedding_search(q, qs, n, field)``.  The
``CosineDistance ... ORDER BY ... LIMIT n`` of pgvector is replaced by the exact HBM index
(``assistant.storage.index``), and ``embedding_search`` accepts a precomputed ``query_embedding``
so callers that already embedded the question do not embed it twice (the reference did).
"""
from __future__ import annotations

import logging
from typing import List, Optional, Tuple

import numpy as np
from assistant.utils.sync import sync_to_async

from assistant.ai.services.ai_service import get_ai_embdedder
from assistant.conf import settings
from assistant.rag.aggregation import aggregate_documents

logger = logging.getLogger(__name__)
_REFILL_ROUNDS = 4


def cosine_similarity(a, b) -> float:
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    den = np.linalg.norm(a) * np.linalg.norm(b)
    return float(a @ b / den) if den else 0.0


def embeddings_similarity(embedding1, embedding2) -> float:
    return cosine_similarity(embedding1, embedding2)


async def get_embedding(text: str) -> List[float]:
    return (await get_ai_embdedder(settings.EMBEDDING_AI_MODEL).embeddings([text]))[0]


async def embedding_search(query: str, qs, max_scores_n: int = 10, top_n: int = 10,
                           query_embedding: Optional[List[float]] = None) -> List[Tuple[object, float]]:
    """Top documents by aggregated question/sentence similarity -> [(Document, score)] best first."""
    from assistant.storage.models import Document

    logger.info("Embedding search for query: %s", query)
    if query_embedding is None:
        query_embedding = await get_embedding(query)
    hits = await _objects_embedding_search(query_embedding, qs, n=max_scores_n * top_n * 10)
    ranked = aggregate_documents([h.distance for h in hits], [h.document_id for h in hits], max_scores_n, top_n)
    if not ranked:
        return []
    docs = await sync_to_async(lambda: Document.objects.in_bulk([d for d, _ in ranked]))()
    return [(docs[d], s) for d, s in ranked if d in docs]


async def embedding_search_documents(query_embedding, qs, n: int = 10):
    return await _objects_embedding_search(query_embedding, qs, n, field="content_embedding")


async def embedding_search_questions(query_embedding, qs, n: int = 10):
    return await _objects_embedding_search(query_embedding, qs, n)


async def embedding_search_sentences(query_embedding, qs, n: int = 10):
    return await _objects_embedding_search(query_embedding, qs, n)


async def _objects_embedding_search(query_embedding, qs, n: int = 10, field: str = "embedding"):
    """The ``n`` rows of ``qs`` nearest to the query, ascending cosine distance, each annotated with
    ``.distance`` exactly like ``qs.annotate(distance=CosineDistance(field, q)).order_by('distance')[:n]``."""
    from assistant.storage.index import MAX_SEARCH_K, get_index_service

    def run():
        svc = get_index_service()
        want = min(n, MAX_SEARCH_K)
        out = []
        for _round in range(_REFILL_ROUNDS):
            hits = svc.search(qs, query_embedding, want, field)
            if not hits:
                return []
            objs = _load_within(qs, [pk for pk, _ in hits])
            out = []
            for pk, dist in hits:
                o = objs.get(pk)
                if o is not None:
                    o.distance = float(dist)
                    out.append(o)
            dropped = [pk for pk, _ in hits if pk not in objs]
            # LIMIT n semantics (reference search_service.py:191-195): n qualifying rows whenever
            # they exist.  Hits the QuerySet rejected mean stale mirrored metadata: re-mirror those
            # rows and search again, over-fetching by what was lost, until n rows qualify or the
            # index has no more candidates under the filter.  The request never grows past the
            # index's largest k (a bigger one fails on gpu_service); at that size every round still
            # repairs the rows it dropped, up to _REFILL_ROUNDS searches.
            if len(out) >= n or not dropped or len(hits) < want:
                break
            svc.refresh_rows(qs.model, dropped, field)
            want = min(max(2 * want, n + len(dropped)), MAX_SEARCH_K)
        return out[:n]

    return await sync_to_async(run)()


def _load_within(qs, pks):
    """{pk: obj} for the hits that still satisfy ``qs``: the QuerySet, not the index's mirrored
    metadata, decides membership (a row whose wiki moved to another bot or whose processing run was
    edited since it was mirrored is dropped here)."""
    try:
        return {o.pk: o for o in qs.filter(pk__in=pks)}
    except (TypeError, AssertionError, NotImplementedError):  # sliced / combined QuerySets
        keep = set(qs.values_list("pk", flat=True))
        return {pk: o for pk, o in qs.model.objects.in_bulk([p for p in pks if p in keep]).items()}
