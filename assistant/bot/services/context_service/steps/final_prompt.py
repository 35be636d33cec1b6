"""Final system instruction with the retrieved context (reference steps/final_prompt.py:7-45).
The wording is shared with the engine's batched RAG path (django_assistant_bot_amd.engine.rag)."""
from assistant.bot.services.context_service.steps.base import ContextProcessingStep, ai_debugger
from assistant.bot.services.context_service.utils import add_system_message
from django_assistant_bot_amd.engine.rag import final_info_message


class FinalPromptStep(ContextProcessingStep):
    debug_info_key = "final"

    @ai_debugger
    async def run(self):
        info = self._state.final_info if self._state.context_is_ok else None
        self._state.messages = add_system_message(self._state.messages,
                                                  final_info_message(info, self._state.user_question))
        self._debug_info["input"] = [f"[{d.id}] {d.name}" for d in (self._state.documents or [])]
