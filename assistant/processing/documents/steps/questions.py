"""Question generation and cross-document de-duplication (reference documents/steps/questions.py).

Generate: per <= 500-char part, the LLM lists every question the part answers (summed length >= half the
part, right language).  Merge: for each question, the nearest question of any EARLIER document; at
cosine distance <= 0.05 the LLM confirms the two ask exactly the same thing and then picks the document
that answers it better -- the other copy is deleted, so retrieval is not split between duplicates."""
from __future__ import annotations

from typing import List

from assistant.processing.documents.steps.base import DocumentProcessingStep
from assistant.processing.utils import expected_language, json_prompt, language_ok, split_text_by_parts
from assistant.utils.repeat_until import repeat_until

PART_CHARS = 500
DUPLICATE_DISTANCE = 0.05


class GenerateQuestionsStep(DocumentProcessingStep):
    ai_model_setting = "QUESTIONS_AI_MODEL"

    @staticmethod
    def prompt(text: str) -> str:
        return ("Here is a piece of a document:\n"
                f"```\n{text.strip()}\n```\n"
                "List every question this text can ANSWER -- and only those whose answers it contains. Use the "
                "text's key terms so that the questions match it well in a search. Write natural sentences without "
                "stray spaces or symbols, in the language of the document.\n"
                f"{json_prompt('document_questions')}")

    async def generate(self, text: str, lang=None) -> List[str]:
        min_len = int(len(text) * 0.5)

        def ok(resp) -> bool:
            q = resp.result.get("questions")
            return (isinstance(q, list) and all(isinstance(x, str) for x in q)
                    and sum(len(x) for x in q) >= min_len and language_ok(q, lang))

        resp = await repeat_until(self._ai.prompt, self.prompt(text), json_format=True, condition=ok)
        return [x.strip() for x in resp.result["questions"] if x.strip()]

    async def run(self):
        path = await self._repo.wiki_path(self._document)
        text = f"# {path.replace(' / ', '. ')}\n\n{self._document.content}\n"
        lang = expected_language(self._document.content)
        questions: List[str] = []
        for part in split_text_by_parts(text, PART_CHARS):
            questions += await self.generate(part, lang)
        await self._repo.add_texts(self._document, "questions", questions)


class MergeQuestionsStep(DocumentProcessingStep):
    ai_model_setting = "QUESTIONS_AI_MODEL"

    async def run(self):
        for q in await self._repo.texts(self._document, "questions"):
            if q.embedding is None:
                continue
            hit = await self._repo.nearest_earlier_question(self._document, q.embedding)
            if hit is None:
                continue
            other, distance = hit
            self._logger.info("question %r ~ %r (distance %.4f)", q.text, other.text, distance)
            if distance <= DUPLICATE_DISTANCE and await self.same_meaning(q.text, other.text):
                await self.merge(q, other)

    async def same_meaning(self, a: str, b: str) -> bool:
        if a == b:
            return True
        prompt = ("Do these two questions ask for exactly the same thing?\n"
                  f"```\n1. {a}\n2. {b}\n```\n\n"
                  "They are the same only if they request identical information with the same goal; any difference "
                  "in context, purpose, level of detail or scope -- however small -- makes them different.\n"
                  "Answer true if they are the same, false otherwise.\n"
                  f"{json_prompt('questions_similarity')}")
        resp = await repeat_until(self._ai.prompt, prompt, json_format=True,
                                  condition=lambda r: isinstance(r.result.get("result"), bool))
        return resp.result["result"]

    async def merge(self, question, other):
        doc_a = await self._repo.document_for(question)
        doc_b = await self._repo.document_for(other)
        path_a = (await self._repo.wiki_path(doc_a)).replace(" / ", ". ")
        path_b = (await self._repo.wiki_path(doc_b)).replace(" / ", ". ")
        prompt = ("Which of the two documents answers this question better?\n"
                  f"```\n{question.text}\n```\n\n"
                  f"1. First document\n```\n# {path_a}\n\n{doc_a.content}\n```\n\n"
                  f"2. Second document\n```\n# {path_b}\n\n{doc_b.content}\n```\n\n"
                  "Answer 1 for the first document or 2 for the second.\n"
                  f"{json_prompt('questions_merge')}")
        resp = await repeat_until(self._ai.prompt, prompt, json_format=True,
                                  condition=lambda r: r.result.get("result") in (1, 2))
        loser = other if resp.result["result"] == 1 else question
        self._logger.info("merged duplicate question; deleting %r of document %s", loser.text,
                          getattr(loser, "document_id", None))
        await self._repo.delete_question(loser)
