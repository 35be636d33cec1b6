"""Single-prompt convenience wrapper around a provider (reference ai/dialog.py:11-45)."""
from __future__ import annotations

import logging
from typing import List

from assistant.ai.domain import AIResponse, Message
from assistant.ai.providers.base import AIProvider, accepts_json_schema
from assistant.ai.services.ai_service import get_ai_provider

logger = logging.getLogger(__name__)


class AIDialog(AIProvider):
    def __init__(self, model: str):
        self._model = model
        self._provider = get_ai_provider(model)

    async def prompt(self, context: str, role: str = "user", *args, **kwargs) -> AIResponse:
        resp = await self._provider.get_response([Message(role=role, content=context)], *args, **kwargs)
        logger.debug("AI response: %s", resp)
        return resp

    @property
    def calls_attempts(self):
        return self._provider.calls_attempts

    @calls_attempts.setter
    def calls_attempts(self, value):
        self._provider.calls_attempts = value

    @property
    def context_size(self) -> int:
        return self._provider.context_size

    def calculate_tokens(self, text: str) -> int:
        return self._provider.calculate_tokens(text)

    async def get_response(self, messages: List[Message], max_tokens: int = 1024,
                           json_format: bool = False, json_schema: dict | None = None) -> AIResponse:
        if json_schema is None or not accepts_json_schema(self._provider.get_response):
            return await self._provider.get_response(messages, max_tokens, json_format or json_schema is not None)
        return await self._provider.get_response(messages, max_tokens, json_format, json_schema=json_schema)
