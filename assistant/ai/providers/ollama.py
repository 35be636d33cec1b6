"""Ollama /api/chat with JSON-mode validation + repair retries (reference ai/providers/ollama.py:16-107)."""
from __future__ import annotations

import json
import logging
import time
from typing import List

from assistant.ai.domain import AIResponse, Message
from assistant.ai.providers._http import post_json
from assistant.ai.providers.base import AIProvider

logger = logging.getLogger(__name__)


class OllamaAIProvider(AIProvider):
    def __init__(self, model: str, host: str, debug=False):
        self._model = model
        self._host = host.rstrip("/")
        if debug:
            self.calls_attempts = []

    @property
    def context_size(self) -> int:
        return 8000

    def calculate_tokens(self, text: str) -> int:
        return len(text.split()) // 2

    @staticmethod
    def _check_roles(messages: List[Message]) -> None:
        for a, b in zip(messages, messages[1:]):
            if a["role"] == b["role"]:
                raise ValueError("OllamaAIProvider does not support consecutive messages of the same role")

    @staticmethod
    def _parse_json(content: str):
        """JSON, or JSON after escaping raw newlines inside strings; None if unparseable/degenerate."""
        if "\t\t\t\t" in content or "\n\n\n\n" in content:
            return None
        try:
            return json.loads(content)
        except json.JSONDecodeError:
            pass
        if "\n" in content and "\\n" not in content:
            try:
                return json.loads(content.replace("\n", "\\n"))
            except json.JSONDecodeError:
                return None
        return None

    async def get_response(self, messages: List[Message], max_tokens: int = 1024,
                           json_format: bool = False, json_schema: dict | None = None) -> AIResponse:
        self._check_roles(messages)
        body = {"model": self._model, "messages": [dict(m) for m in messages], "stream": False,
                "options": {"num_predict": max_tokens}}
        if json_schema is not None:
            body["format"] = json_schema  # Ollama structured outputs
            json_format = True
        elif json_format:
            body["format"] = "json"
        t0 = time.time()
        for attempt in range(1, 6):
            data = await post_json(f"{self._host}/api/chat", body)
            logger.debug("raw Ollama response (%.2f s): %s", time.time() - t0, data)
            content = data["message"]["content"]
            if json_format:
                result = self._parse_json(content)
                if result is None:
                    logger.warning("unparseable JSON from Ollama (attempt %d), retrying", attempt)
                    continue
            else:
                result = content.strip()
            self._record_attempts(attempt)
            return AIResponse(result=result,
                              usage={"model": data.get("model", self._model),
                                     "prompt_tokens": data.get("prompt_eval_count", 0),
                                     "completion_tokens": data.get("eval_count", 0)},
                              length_limited=not data.get("done", True))
        raise ValueError("Failed to parse JSON response")
