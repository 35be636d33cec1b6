"""Retrieval step (reference steps/embeddings.py:11-77): related questions + broad document search.

One query embedding serves both searches (the reference embedded the question twice)."""
from __future__ import annotations

from assistant.bot.services.context_service.steps.base import ContextProcessingStep, time_debugger
from assistant.rag.knowledge import get_knowledge_base
from assistant.rag.services.search_service import get_embedding
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
        kb = get_knowledge_base(self._bot)
        query = self._state.user_question
        q_emb = await get_embedding(query)
        questions = await kb.related_questions(q_emb, self.related_n)
        self._state.related_questions = questions
        self._debug_info["related_questions"] = [f"[{q.id} {1 - q.distance}] {q.text}" for q in questions[:5]]
        if questions and questions[0].distance < SAME_QUESTION_DISTANCE:
            self._debug_info["the_same_question"] = questions[0].text
            doc = await kb.get_document(questions[0].document_id)
            documents = [(doc, 1 - questions[0].distance)] if doc is not None else []
        else:
            documents = await kb.search_documents(query, q_emb, max_scores_n=self.max_scores_n, top_n=self.top_n)
        unique = list({d.id: (d, s) for d, s in documents}.values())
        self._debug_info["documents"] = [f"[{d.id} {s}] {d.name}" for d, s in unique]
        self._state.documents = [d for d, _ in unique]
