"""Persistence seam of the ingest pipeline.

The reference steps read and write the ORM directly (reference processing/wiki.py:29-46,
documents/steps/*.py).  Here they go through an ``IngestRepository``: ``DjangoIngestRepository`` in
production (Celery tasks), ``MemoryIngestRepository`` for tests, notebooks and the offline bulk
ingest (``benchmarks``), which keeps the same record attributes as the models (``document.content``,
``question.text``, ``question.embedding`` ...) and searches question embeddings with the engine's
exact ``VectorIndex``.
"""
from __future__ import annotations

import dataclasses
import itertools
from abc import ABC, abstractmethod
from typing import Dict, Optional, Sequence, Tuple

from assistant.utils.sync import sync_to_async


class IngestRepository(ABC):
    @abstractmethod
    async def start_processing(self, wiki): ...

    @abstractmethod
    async def add_document(self, processing, wiki, name: str, content: str): ...

    @abstractmethod
    async def wiki_path(self, document) -> str: ...

    @abstractmethod
    async def save_document_content(self, document) -> None: ...

    @abstractmethod
    async def add_texts(self, document, kind: str, texts: Sequence[str]) -> None:
        """kind: 'sentences' | 'questions'; ``order`` is the position in the document."""

    @abstractmethod
    async def texts(self, document, kind: str) -> list: ...

    @abstractmethod
    async def set_embeddings(self, rows: list, kind: str, vectors: Sequence[Sequence[float]]) -> None: ...

    @abstractmethod
    async def nearest_earlier_question(self, document, embedding) -> Optional[Tuple[object, float]]:
        """Nearest question (cosine distance) among documents with a smaller id."""

    @abstractmethod
    async def delete_question(self, question) -> None: ...

    @abstractmethod
    async def document_for(self, question): ...

    @abstractmethod
    async def finalize(self, processing) -> None:
        """Mark the run completed and drop older runs of the same wiki (with their documents)."""


# ------------------------------------------------------------------------------------------ memory

@dataclasses.dataclass
class MemWiki:
    id: int
    title: str
    content: str
    path: str = ""
    bot_codename: str = "default"

    def __post_init__(self):
        self.path = self.path or self.title


@dataclasses.dataclass
class MemProcessing:
    id: int
    wiki: MemWiki
    status: str = "in_progress"


@dataclasses.dataclass
class MemDocument:
    id: int
    processing: MemProcessing
    wiki: MemWiki
    name: str
    content: str

    @property
    def wiki_id(self):
        return self.wiki.id


@dataclasses.dataclass
class MemText:
    id: int
    document: MemDocument
    text: str
    order: int
    embedding: Optional[list] = None


class MemoryIngestRepository(IngestRepository):
    def __init__(self):
        self._ids = itertools.count(1)
        self.processings: Dict[int, MemProcessing] = {}
        self.documents: Dict[int, MemDocument] = {}
        self.rows: Dict[str, Dict[int, MemText]] = {"sentences": {}, "questions": {}}

    async def start_processing(self, wiki):
        p = MemProcessing(next(self._ids), wiki)
        self.processings[p.id] = p
        return p

    async def add_document(self, processing, wiki, name, content):
        d = MemDocument(next(self._ids), processing, wiki, name, content)
        self.documents[d.id] = d
        return d

    async def wiki_path(self, document):
        return document.wiki.path

    async def save_document_content(self, document):
        return None

    async def add_texts(self, document, kind, texts):
        for i, t in enumerate(texts):
            r = MemText(next(self._ids), document, t, i)
            self.rows[kind][r.id] = r

    async def texts(self, document, kind):
        return [r for r in self.rows[kind].values() if r.document is document]

    async def set_embeddings(self, rows, kind, vectors):
        for r, v in zip(rows, vectors):
            r.embedding = list(v)

    async def nearest_earlier_question(self, document, embedding):
        import numpy as np

        cands = [q for q in self.rows["questions"].values()
                 if q.document.id < document.id and q.embedding is not None and q.document.id in self.documents]
        if not cands:
            return None
        m = np.asarray([q.embedding for q in cands], dtype=np.float64)
        e = np.asarray(embedding, dtype=np.float64)
        sims = m @ e / (np.linalg.norm(m, axis=1) * np.linalg.norm(e) + 1e-12)
        i = int(np.argmax(sims))
        return cands[i], float(1.0 - sims[i])

    async def delete_question(self, question):
        self.rows["questions"].pop(question.id, None)

    async def document_for(self, question):
        return question.document

    async def finalize(self, processing):
        processing.status = "completed"
        for pid, p in list(self.processings.items()):
            if p.wiki is processing.wiki and p is not processing:
                del self.processings[pid]
                for did, d in list(self.documents.items()):
                    if d.processing is p:
                        del self.documents[did]
                        for kind in self.rows:
                            for rid, r in list(self.rows[kind].items()):
                                if r.document is d:
                                    del self.rows[kind][rid]


# ------------------------------------------------------------------------------------------ django

class DjangoIngestRepository(IngestRepository):
    """ORM persistence (reference processing/wiki.py, documents/steps/*.py, tasks.py:59-74)."""

    async def start_processing(self, wiki):
        from assistant.storage.models import WikiDocumentProcessing
        return await sync_to_async(WikiDocumentProcessing.objects.create)(wiki_document=wiki)

    async def add_document(self, processing, wiki, name, content):
        from assistant.storage.models import Document
        return await sync_to_async(Document.objects.create)(processing=processing, name=name, content=content,
                                                            wiki=wiki)

    async def wiki_path(self, document):
        return await sync_to_async(lambda: document.wiki.path if document.wiki_id else document.name)()

    async def save_document_content(self, document):
        await sync_to_async(document.save)(update_fields=["content"])

    def _model(self, kind):
        from assistant.storage.models import Question, Sentence
        return {"sentences": Sentence, "questions": Question}[kind]

    async def add_texts(self, document, kind, texts):
        model = self._model(kind)
        rows = [model(document=document, text=t, order=i) for i, t in enumerate(texts)]
        await sync_to_async(model.objects.bulk_create)(rows)

    async def texts(self, document, kind):
        model = self._model(kind)
        return await sync_to_async(lambda: list(model.objects.filter(document=document).order_by("order", "id")))()

    async def set_embeddings(self, rows, kind, vectors):
        model = self._model(kind)
        for r, v in zip(rows, vectors):
            r.embedding = list(v)

        def save():
            from assistant.storage.index import get_index_service

            model.objects.bulk_update(rows, fields=["embedding"])
            get_index_service().upsert_objects(model, rows, "embedding")  # bulk_update fires no signals
        await sync_to_async(save)()

    async def nearest_earlier_question(self, document, embedding):
        from assistant.rag.services.search_service import embedding_search_questions
        from assistant.storage.models import Question

        from assistant.storage.index import with_index_filter

        qs = with_index_filter(Question.objects.filter(document__id__lt=document.id), doc_lt=document.id)
        hits = await embedding_search_questions(embedding, qs, n=1)
        return (hits[0], float(hits[0].distance)) if hits else None

    async def delete_question(self, question):
        await sync_to_async(question.delete)()

    async def document_for(self, question):
        return await sync_to_async(lambda: question.document)()

    async def finalize(self, processing):
        from django.db import transaction

        from assistant.storage.models import WikiDocumentProcessing

        def run():
            from assistant.storage.index import get_index_service

            with transaction.atomic():
                processing.status = WikiDocumentProcessing.Status.COMPLETED
                processing.save(update_fields=["status"])
                processing.wiki_document.processing.exclude(id=processing.id).delete()
            # the wiki's rows now match the COMPLETED filter: re-mirror their group bit
            get_index_service().refresh_wiki(processing.wiki_document_id)
        await sync_to_async(run)()
