"""Groq (OpenAI-compatible API) with a shared 2 s throttle and JSON-mode retries
(reference ai/providers/groq.py:18-132)."""
from __future__ import annotations

import json
import logging
from typing import List

from assistant.ai.domain import AIResponse, Message
from assistant.ai.providers._http import HTTPError
from assistant.ai.providers.openai import ChatGPTAIProvider
from assistant.utils.throttle import Throttle

logger = logging.getLogger(__name__)


class GroqAIProvider(ChatGPTAIProvider):
    _throttle = Throttle(2)  # shared by every instance: Groq's per-key rate limit

    def __init__(self, model: str, api_key: str, base_url: str = "https://api.groq.com/openai/v1", debug=False):
        super().__init__(model, api_key, base_url)
        if debug:
            self.calls_attempts = []

    async def get_response(self, messages: List[Message], max_tokens: int = 1024,
                           json_format: bool = False, json_schema: dict | None = None) -> AIResponse:
        json_format = json_format or json_schema is not None
        converted = [self.convert_message(m) for m in messages]
        if any(isinstance(m["content"], list) for m in converted):
            converted = [m for m in converted if m["role"] != "system"]  # vision models reject system turns
        body = {"model": self._model, "messages": converted, "max_tokens": max_tokens}
        if json_format:
            body["response_format"] = {"type": "json_object"}
        for attempt in range(1, 6):
            await self._throttle()
            try:
                data = await self._call(body)
            except HTTPError as exc:
                if json_format and exc.status == 400 and "json" in exc.body.lower():
                    logger.warning("Groq JSON validation failed (attempt %d), retrying", attempt)
                    continue
                raise
            choice = data["choices"][0]
            content = choice["message"].get("content") or ""
            try:
                result = json.loads(content) if json_format else content.strip()
            except json.JSONDecodeError:
                logger.warning("invalid JSON from Groq (attempt %d), retrying", attempt)
                continue
            usage = data.get("usage") or {}
            self._record_attempts(attempt)
            return AIResponse(result=result,
                              usage={"model": data.get("model", self._model),
                                     "prompt_tokens": usage.get("prompt_tokens", 0),
                                     "completion_tokens": usage.get("completion_tokens", 0)},
                              length_limited=choice.get("finish_reason") == "length")
        raise ValueError("Failed to parse JSON response")
