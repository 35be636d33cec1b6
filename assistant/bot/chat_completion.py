"""Strong-model answer generation over the enriched context (reference bot/chat_completion.py:16-45)."""
from __future__ import annotations

import logging

from assistant.ai.domain import AIResponse
from assistant.ai.providers.base import AIDebugger
from assistant.ai.services.ai_service import get_ai_provider
from assistant.bot.services.context_service.service import ContextService

logger = logging.getLogger(__name__)


class ChatCompletion:
    context_service_class = ContextService

    def __init__(self, bot, resource_manager, fast_ai_model: str, strong_ai_model: str):
        self.bot = bot
        self.resource_manager = resource_manager
        self.fast_ai_model = fast_ai_model
        self.strong_ai_model = strong_ai_model

    async def generate_answer(self, messages: list, debug_info: dict = None, do_interrupt=None,
                              max_tokens: int = 1024) -> AIResponse:
        debug_info = debug_info if debug_info is not None else {}
        if messages:
            debug_info["query"] = messages[-1]["content"]
        service = self.context_service_class(bot=self.bot, fast_ai_model=self.fast_ai_model,
                                             strong_ai_model=self.strong_ai_model, messages=messages,
                                             debug_info=debug_info, do_interrupt=do_interrupt)
        enriched = await service.enrich()
        strong_ai = get_ai_provider(self.strong_ai_model)
        with AIDebugger(strong_ai, debug_info, "final"):
            return await strong_ai.get_response(enriched, max_tokens=max_tokens)
