"""Topic classification with the fast model (reference steps/classify.py:13-97)."""
from __future__ import annotations

from assistant.ai.providers.base import accepts_json_schema
from assistant.bot.services.context_service.steps.base import ContextProcessingStep, ai_debugger
from assistant.bot.services.context_service.utils import add_system_message, get_list_str
from assistant.bot.services.schema_service import json_prompt
from assistant.rag.knowledge import get_knowledge_base
from assistant.utils.fuzzy import extract_bests
from assistant.utils.repeat_until import repeat_until

SMALL_TALK = "Small talk"


class ClassifyStep(ContextProcessingStep):
    debug_info_key = "classify"
    _offtopic_examples = [("Hello", SMALL_TALK), ("How are you?", SMALL_TALK),
                          ("What's the weather in Moscow?", SMALL_TALK)]

    @ai_debugger
    async def run(self):
        kb = get_knowledge_base(self._bot)
        roots = await kb.topics()
        if not roots:  # empty knowledge base: nothing to route to, skip the LLM call
            self._debug_info["topic"] = SMALL_TALK
            return
        topics = [SMALL_TALK] + [t.title for t in roots]
        examples = self._offtopic_examples + [(q, t.title) for t in roots for q in t.examples]
        messages = add_system_message(self._state.messages, self.prompt(topics, examples, self._state.user_question))
        # providers that enforce JSON Schemas (the MI355X engine: constrained decoding) answer with
        # one of the topic titles in one generation; the others keep the reference's retry loop
        kw = {"json_schema": self.schema(topics)} if accepts_json_schema(self._fast_ai.get_response) else {}
        response = await repeat_until(self._fast_ai.get_response, messages, max_tokens=256, json_format=True,
                                      condition=self._condition, **kw)
        topic = response.result["topic"]
        self._logger.info("classified question as %s", topic)
        best = extract_bests(topic, topics, limit=1)
        best_title = best[0][0] if best else SMALL_TALK
        if best_title == SMALL_TALK:
            self._debug_info["topic"] = SMALL_TALK
            return
        chosen = roots[topics.index(best_title) - 1]
        self._debug_info["topic"] = chosen.title
        self._state.topic = chosen

    @staticmethod
    def schema(topics) -> dict:
        return {"type": "object", "properties": {"topic": {"type": "string", "enum": list(topics)}},
                "required": ["topic"]}

    @staticmethod
    def prompt(topics, examples, user_question) -> str:
        return (
            "Classify the user's question in a way that will help to search answer in the database by sentence "
            "embeddings.\nDo not answer the question, but just classify to provide the search query.\n\n"
            f"Possible topics:\n{get_list_str(topics)}\n"
            f"Examples:\n{get_list_str([f'{chr(34)}{q}{chr(34)} -> {chr(34)}{t}{chr(34)}' for q, t in examples])}\n\n"
            f"Please, provide the topic name that is relevant to the user question:\n```\n{user_question}\n```\n"
            "Give only the topic name in the original spelling including language.\n"
            f"{json_prompt(['classify'])}"
        )

    @staticmethod
    def _condition(response) -> bool:
        return isinstance(response.result, dict) and isinstance(response.result.get("topic"), str)
