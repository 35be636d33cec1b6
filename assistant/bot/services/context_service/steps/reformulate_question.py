"""Optional: rewrite the question into a search query (reference steps/reformulate_question.py:7-33)."""
from assistant.bot.services.context_service.steps.base import ContextProcessingStep, ai_debugger
from assistant.bot.services.context_service.utils import add_system_message
from assistant.bot.services.schema_service import json_prompt
from assistant.utils.repeat_until import repeat_until


class ReformulateQuestionStep(ContextProcessingStep):
    debug_info_key = "reformulate_question"

    @ai_debugger
    async def run(self):
        messages = add_system_message(self._state.messages, (
            "Reformulate the user's question in a way that will help to search answer in the database by sentence "
            "embeddings.\nDo not answer the question, but just reformulate to provide the search query.\n"
            "You must use the original query language.\n"
            f"{json_prompt(['reformulate'])}"))
        resp = await repeat_until(self._fast_ai.get_response, messages, max_tokens=256, json_format=True,
                                  condition=lambda r: isinstance(r.result, dict) and isinstance(r.result.get("query"),
                                                                                                str))
        query = resp.result["query"]
        self._logger.info("reformulated question: %s", query)
        self._debug_info["new_question"] = query
        self._state.user_question = query
