"""Embedding steps (reference documents/steps/embeddings.py:14-90): one embedder call per document
with all its sentences / questions (the engine-backed embedders batch them into packed varlen encoder
passes), one vector per text, written back in bulk."""
from __future__ import annotations

from assistant.ai.services.ai_service import get_ai_embdedder
from assistant.conf import settings
from assistant.processing.documents.steps.base import DocumentProcessingStep


class _RowsEmbeddingsStep(DocumentProcessingStep):
    kind: str = None

    def __init__(self, document, repository):
        super().__init__(document, repository)
        self._embedder = get_ai_embdedder(settings.EMBEDDING_AI_MODEL)

    async def run(self):
        rows = await self._repo.texts(self._document, self.kind)
        if not rows:
            return
        vectors = await self._embedder.embeddings([r.text for r in rows])
        if len(vectors) != len(rows) or any(len(v) == 0 for v in vectors):
            raise RuntimeError(f"embedder returned {len(vectors)} vectors for {len(rows)} {self.kind}")
        await self._repo.set_embeddings(rows, self.kind, vectors)


class SentencesEmbeddingsStep(_RowsEmbeddingsStep):
    kind = "sentences"


class QuestionsEmbeddingsStep(_RowsEmbeddingsStep):
    kind = "questions"


class ContentEmbeddingsStep(DocumentProcessingStep):
    """Whole-document embedding (not in the default pipeline, as in the reference)."""

    async def run(self):
        emb = (await get_ai_embdedder(settings.EMBEDDING_AI_MODEL).embeddings([self._document.content]))[0]
        self._document.content_embedding = emb
        save = getattr(self._document, "save", None)
        if save is not None:
            from assistant.utils.sync import sync_to_async
            await sync_to_async(save)(update_fields=["content_embedding"])
