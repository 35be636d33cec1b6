"""Sentence extraction for sentence-level retrieval (reference documents/steps/sentences.py:19-119).

The section (prefixed with its wiki path) is cut into <= 500-character newline-bounded parts; each part
is split into standalone sentences by the LLM, validated for coverage (summed length >=
min(5 x words, 0.8 x chars)) and language.  ``order`` is the sentence's position in the document (the
reference always stored 0)."""
from __future__ import annotations

from typing import List

from assistant.processing.documents.steps.base import DocumentProcessingStep
from assistant.processing.utils import estimated_min_length, expected_language, language_ok, split_text_by_parts
from assistant.utils.repeat_until import repeat_until

PART_CHARS = 500


def sentences_prompt(text: str) -> str:
    return ("Split the text below into self-contained sentences; they will be embedded for semantic search:\n"
            f"```\n{text.strip()}\n```\n"
            "Together the sentences must cover the whole text -- leave nothing out. Strip formatting and stray "
            "symbols but keep natural punctuation, so each sentence reads on its own. Write in the language of the "
            "text.\n"
            "Answer with JSON exactly like:\n```json\n{\n  \"sentences\": [\n    \"First sentence.\",\n"
            "    \"Second sentence.\"\n  ]\n}\n```\n")


async def split_text_to_sentences(text: str, ai, lang=None) -> List[str]:
    min_len = estimated_min_length(text)

    def ok(resp) -> bool:
        s = resp.result.get("sentences")
        return (isinstance(s, list) and all(isinstance(x, str) for x in s)
                and sum(len(x) for x in s) >= min_len and language_ok(s, lang))

    resp = await repeat_until(ai.prompt, sentences_prompt(text), json_format=True, condition=ok)
    return [x.strip() for x in resp.result["sentences"] if x.strip()]


class ExtractSentencesStep(DocumentProcessingStep):
    ai_model_setting = "SENTENCES_AI_MODEL"

    async def run(self):
        path = await self._repo.wiki_path(self._document)
        text = f"# {path}\n\n{self._document.content}\n"
        lang = expected_language(self._document.content)
        sentences: List[str] = []
        for part in split_text_by_parts(text, PART_CHARS):
            sentences += await split_text_to_sentences(part, self._ai, lang)
        await self._repo.add_texts(self._document, "sentences", sentences)
