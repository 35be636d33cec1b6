"""OpenAI chat completions over the REST API (reference ai/providers/openai.py:13-63)."""
from __future__ import annotations

import json
import logging
import time
from typing import List

from assistant.ai.domain import AIResponse, Message
from assistant.ai.providers._http import post_json
from assistant.ai.providers.base import AIProvider

logger = logging.getLogger(__name__)


class ChatGPTAIProvider(AIProvider):
    def __init__(self, model: str, api_key: str, base_url: str = "https://api.openai.com/v1"):
        self._model = model
        self._api_key = api_key
        self._base_url = base_url.rstrip("/")

    @property
    def context_size(self) -> int:
        return 8000

    def calculate_tokens(self, text: str) -> int:
        return len(text.split()) // 2

    def _payload(self, messages, max_tokens, json_format, json_schema=None):
        body = {"model": self._model, "messages": [self.convert_message(m) for m in messages],
                "max_tokens": max_tokens}
        if json_schema is not None:
            body["response_format"] = {"type": "json_schema",
                                       "json_schema": {"name": "response", "schema": json_schema}}
        elif json_format:
            body["response_format"] = {"type": "json_object"}
        return body

    @staticmethod
    def convert_message(message: Message) -> dict:
        if message.get("images"):
            parts = [{"type": "text", "text": message["content"]}] if message.get("content") else []
            parts += [{"type": "image_url", "image_url": {"url": f"data:image/jpeg;base64,{img}"}}
                      for img in message["images"]]
            return {"role": message["role"], "content": parts}
        return {"role": message["role"], "content": message["content"]}

    async def _call(self, body: dict) -> dict:
        return await post_json(f"{self._base_url}/chat/completions", body,
                               headers={"Authorization": f"Bearer {self._api_key}"})

    async def get_response(self, messages: List[Message], max_tokens: int = 1024,
                           json_format: bool = False, json_schema: dict | None = None) -> AIResponse:
        t0 = time.time()
        json_format = json_format or json_schema is not None
        data = await self._call(self._payload(messages, max_tokens, json_format, json_schema))
        logger.debug("raw completion (%.2f s): %s", time.time() - t0, data)
        choice = data["choices"][0]
        content = choice["message"].get("content") or ""
        result = json.loads(content) if json_format else content.strip()
        usage = data.get("usage") or {}
        self._record_attempts(1)
        return AIResponse(result=result,
                          usage={"model": data.get("model", self._model),
                                 "prompt_tokens": usage.get("prompt_tokens", 0),
                                 "completion_tokens": usage.get("completion_tokens", 0)},
                          length_limited=choice.get("finish_reason") == "length")
