"""Knowledge-base seam of the context pipeline.

The reference's context steps query the ORM directly (topics = root ``WikiDocument``s, related
questions / broad search over ``Question`` embeddings, reference steps/classify.py:17-97,
steps/embeddings.py:11-77).  The steps here go through ``KnowledgeBase``:

  * ``DjangoKnowledgeBase(bot)`` -- production: ORM rows, index search through
    ``assistant.storage.index`` (the HBM-resident VectorIndex or the gpu_service index).
  * ``MemoryKnowledgeBase``   -- documents + questions held in process, searched with the engine's
    ``VectorIndex`` (native MFMA score GEMM + radix top-k on a GPU, torch reference on CPU).  Used by
    tests, the in-memory console and benchmarks; needs no database.

``get_knowledge_base(bot)`` returns ``bot.knowledge`` when the bot record carries one, else the
Django implementation.
"""
from __future__ import annotations

import dataclasses
import random
from abc import ABC, abstractmethod
from typing import Dict, List, Optional, Sequence, Tuple

from assistant.rag.aggregation import aggregate_documents
from assistant.utils.sync import sync_to_async

try:
    import torch
except ImportError:  # pragma: no cover - the memory knowledge base needs torch; Django paths do not
    torch = None


@dataclasses.dataclass
class Topic:
    id: int
    title: str
    examples: List[str] = dataclasses.field(default_factory=list)


@dataclasses.dataclass
class WikiRef:
    path: str
    id: Optional[int] = None


@dataclasses.dataclass
class KnowledgeDocument:
    id: int
    name: str
    content: str
    wiki: Optional[WikiRef] = None
    topic_id: Optional[int] = None

    @property
    def wiki_id(self):
        return self.wiki.id if self.wiki else None


@dataclasses.dataclass
class QuestionHit:
    id: int
    text: str
    document_id: int
    distance: float


class KnowledgeBase(ABC):
    @abstractmethod
    async def topics(self, examples_per_topic: int = 2) -> List[Topic]: ...

    @abstractmethod
    async def related_questions(self, embedding, n: int) -> List[QuestionHit]: ...

    @abstractmethod
    async def search_documents(self, query: str, embedding, max_scores_n: int,
                               top_n: int) -> List[Tuple[object, float]]: ...

    @abstractmethod
    async def get_document(self, doc_id) -> Optional[object]: ...


class EmptyKnowledgeBase(KnowledgeBase):
    """No documents: every question is answered without retrieved context."""

    async def topics(self, examples_per_topic: int = 2):
        return []

    async def related_questions(self, embedding, n):
        return []

    async def search_documents(self, query, embedding, max_scores_n, top_n):
        return []

    async def get_document(self, doc_id):
        return None


def get_knowledge_base(bot) -> KnowledgeBase:
    kb = getattr(bot, "knowledge", None)
    return kb if kb is not None else DjangoKnowledgeBase(bot)


# ------------------------------------------------------------------------------------------- memory

class MemoryKnowledgeBase(KnowledgeBase):
    """Question-level index over in-process documents (same broad-search semantics as the Django
    path: k = max_scores_n * top_n * 10 nearest questions, aggregated per document)."""

    def __init__(self, embed_fn, dim: int, device=None):
        from django_assistant_bot_amd.engine.vector_index import VectorIndex

        self._embed = embed_fn  # async (List[str]) -> List[List[float]]
        self.index = VectorIndex(dim, device=device, capacity=1024)
        self.documents: Dict[int, KnowledgeDocument] = {}
        self.questions: Dict[int, Tuple[str, int]] = {}
        self._topics: Dict[int, str] = {}
        self._next_q = 1

    async def add_document(self, doc: KnowledgeDocument, questions: Sequence[str], topic: Optional[str] = None):
        if topic is not None:
            tid = next((i for i, t in self._topics.items() if t == topic), None)
            if tid is None:
                tid = len(self._topics) + 1
                self._topics[tid] = topic
            doc.topic_id = tid
        self.documents[doc.id] = doc
        questions = list(questions)
        if not questions:
            return
        vecs = await self._embed(questions)
        ids = list(range(self._next_q, self._next_q + len(questions)))
        self._next_q += len(questions)
        for qid, text in zip(ids, questions):
            self.questions[qid] = (text, doc.id)
        self.index.add(ids, vecs, doc_ids=[doc.id] * len(ids))

    async def topics(self, examples_per_topic: int = 2) -> List[Topic]:
        out = []
        for tid, title in self._topics.items():
            qs = [t for t, d in self.questions.values() if self.documents[d].topic_id == tid]
            out.append(Topic(tid, title, random.sample(qs, min(examples_per_topic, len(qs)))))
        return out

    def _search(self, embedding, k: int) -> List[QuestionHit]:
        sims, ids, docs = self.index.search([list(embedding)], k)
        hits = []
        for s, i, d in zip(sims[0].tolist(), ids[0].tolist(), docs[0].tolist()):
            if i < 0:
                continue
            hits.append(QuestionHit(i, self.questions[i][0], d, 1.0 - s))
        return hits

    async def related_questions(self, embedding, n: int) -> List[QuestionHit]:
        return self._search(embedding, n)

    async def search_documents(self, query, embedding, max_scores_n, top_n):
        # broad search: (similarity, document) of the k nearest questions in ONE device->host copy,
        # then the native per-document aggregation -- no per-hit Python objects
        sims, ids, docs = self.index.search([list(embedding)], max_scores_n * top_n * 10)
        sd = torch.stack([sims[0].double(), docs[0].double()]).cpu().numpy()
        live = ids[0].cpu().numpy() >= 0 if sims.is_cuda else ids[0].numpy() >= 0
        ranked = aggregate_documents(1.0 - sd[0][live], sd[1][live].astype("int64"), max_scores_n, top_n)
        return [(self.documents[d], s) for d, s in ranked if d in self.documents]

    async def get_document(self, doc_id):
        try:
            return self.documents.get(int(doc_id))
        except (TypeError, ValueError):
            return None


# ------------------------------------------------------------------------------------------- django

class DjangoKnowledgeBase(KnowledgeBase):
    def __init__(self, bot):
        self.bot = bot

    def _completed_questions(self):
        from assistant.storage.index import with_index_filter
        from assistant.storage.models import Question, WikiDocumentProcessing
        qs = Question.objects.filter(document__wiki__bot=self.bot,
                                     document__wiki__processing__status=WikiDocumentProcessing.Status.COMPLETED)
        return with_index_filter(qs, bot=self.bot, completed=True)  # one group compare in the index

    async def topics(self, examples_per_topic: int = 2) -> List[Topic]:
        from assistant.storage.models import Question, WikiDocument, WikiDocumentProcessing

        def load():
            roots = list(WikiDocument.objects.filter(
                bot=self.bot, processing__status=WikiDocumentProcessing.Status.COMPLETED, parent=None).distinct())
            out = []
            for w in roots:
                qs = Question.objects.filter(document__wiki__tree_id=w.tree_id, document__wiki__lft__gte=w.lft,
                                             document__wiki__rght__lte=w.rght).order_by("?")[:examples_per_topic]
                out.append(Topic(w.id, w.title, [q.text for q in qs]))
            return out
        return await sync_to_async(load)()

    async def related_questions(self, embedding, n: int) -> List[QuestionHit]:
        from assistant.rag.services.search_service import embedding_search_questions

        rows = await embedding_search_questions(embedding, self._completed_questions(), n=n)
        return [QuestionHit(q.id, q.text, q.document_id, q.distance) for q in rows]

    async def search_documents(self, query, embedding, max_scores_n, top_n):
        from assistant.rag.services.search_service import embedding_search

        return await embedding_search(query, self._completed_questions(), max_scores_n=max_scores_n, top_n=top_n,
                                      query_embedding=embedding)

    async def get_document(self, doc_id):
        from assistant.storage.models import Document
        return await sync_to_async(lambda: Document.objects.select_related("wiki").filter(id=doc_id).first())()
