"""Known-question matching with the fast model (reference steps/choose_known_question.py:9-61)."""
from __future__ import annotations

from assistant.ai.providers.base import accepts_json_schema
from assistant.bot.services.context_service.steps.base import ContextProcessingStep, ai_debugger
from assistant.bot.services.context_service.utils import add_system_message, get_numerical_list_str
from assistant.bot.services.schema_service import json_prompt
from assistant.rag.knowledge import get_knowledge_base
from assistant.utils.repeat_until import repeat_until


class ChooseKnownQuestionStep(ContextProcessingStep):
    debug_info_key = "known_question_choice"

    @staticmethod
    def prompt(user_question: str, questions: list) -> str:
        return (
            f"The user asked a question:\n```\n{user_question}\n```\n\n"
            "Your task is to determine if any of the known questions below have the same meaning as the user's "
            "question. Two questions have the same meaning if the answer to the user's question would also correctly "
            "answer the known question. Only consider questions to be the same if their answers would be identical.\n"
            f"Here are the known questions:\n```\n{get_numerical_list_str(questions)}\n```\n"
            "Please provide the number of the known question that matches the user's question in meaning. "
            "If none of the known questions match the user's question in meaning, provide `null`.\n"
            f"{json_prompt(['choose_known_question'])}"
        )

    @staticmethod
    def schema(n_questions: int) -> dict:
        """The answer the condition below accepts: the number of a listed question, or null."""
        return {"type": "object", "properties": {"question": {"anyOf": [
            {"type": "integer", "minimum": 1, "maximum": max(1, n_questions)}, {"type": "null"}]}},
            "required": ["question"]}

    @staticmethod
    def _condition(resp) -> bool:
        return isinstance(resp.result, dict) and "question" in resp.result and (
            resp.result["question"] is None or isinstance(resp.result["question"], int))

    @ai_debugger
    async def run(self):
        questions = list(self._state.related_questions or [])[:5]
        if not questions:
            self._debug_info["the_same_question"] = None
            return
        messages = add_system_message([], self.prompt(self._state.user_question, [q.text for q in questions]))
        kw = ({"json_schema": self.schema(len(questions))} if accepts_json_schema(self._fast_ai.get_response)
              else {})
        response = await repeat_until(self._fast_ai.get_response, messages, json_format=True,
                                      condition=self._condition, **kw)
        n = response.result["question"]
        if n and 1 <= n <= len(questions):
            q = questions[n - 1]
            self._debug_info["the_same_question"] = q.text
            document = await get_knowledge_base(self._bot).get_document(q.document_id)
            if document is None:
                return
            self._debug_info["document"] = f"[{document.id}] {document.name}"
            self._state.documents = [document]
        else:
            self._debug_info["the_same_question"] = None
