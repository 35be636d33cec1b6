"""Retrieval step (reference steps/embeddings.py:11-77): related questions + broad document search.

One query embedding serves both searches (the reference embedded the question twice)."""
from __future__ import annotations

from asgiref.sync import sync_to_async

from assistant.bot.services.context_service.steps.base import ContextProcessingStep, time_debugger
from assistant.rag.services.search_service import embedding_search, embedding_search_questions, get_embedding
from assistant.utils.debug import TimeDebugger

SAME_QUESTION_DISTANCE = 0.05


class EmbeddingsStep(ContextProcessingStep):
    debug_info_key = "embedding_search"
    debugger_class = TimeDebugger
    related_n = 5
    max_scores_n = 5
    top_n = 5

    @time_debugger
    async def run(self):
        from assistant.storage.models import Document, Question, WikiDocumentProcessing

        query = self._state.user_question
        q_emb = await get_embedding(query)
        qs = Question.objects.filter(document__wiki__bot=self._bot,
                                     document__wiki__processing__status=WikiDocumentProcessing.Status.COMPLETED)
        questions = list(await embedding_search_questions(q_emb, qs, n=self.related_n))
        self._state.related_questions = questions
        self._debug_info["related_questions"] = [f"[{q.id} {1 - q.distance}] {q.text}" for q in questions[:5]]
        if questions and questions[0].distance < SAME_QUESTION_DISTANCE:
            self._debug_info["the_same_question"] = questions[0].text
            doc = await sync_to_async(lambda: Document.objects.get(id=questions[0].document_id))()
            documents = [(doc, 1 - questions[0].distance)]
        else:
            documents = await embedding_search(query, qs, max_scores_n=self.max_scores_n, top_n=self.top_n,
                                               query_embedding=q_emb)
        unique = list({d.id: (d, s) for d, s in documents}.values())
        self._debug_info["documents"] = [f"[{d.id} {s}] {d.name}" for d, s in unique]
        self._state.documents = [d for d, _ in unique]
