"""Client of the gpu_service ``POST /dialog/`` endpoint (reference ai/providers/gpu_service.py:9-41).

Unlike the reference client, ``max_tokens`` and ``json_format`` are forwarded (the reference dropped
them, so the server always used 1024 / text mode -- SURVEY.md 7.5)."""
from __future__ import annotations

from typing import List

from assistant.ai.domain import AIResponse, Message
from assistant.ai.providers._http import HTTPError, post_json
from assistant.ai.providers.base import AIProvider


class GPUServiceProvider(AIProvider):
    def __init__(self, base_url: str, model: str):
        self._base_url = base_url.rstrip("/")
        self._model = model

    @property
    def context_size(self) -> int:
        return 8000

    def calculate_tokens(self, text: str) -> int:
        return len(text.split()) // 2

    async def get_response(self, messages: List[Message], max_tokens: int = 1024,
                           json_format: bool = False, json_schema: dict | None = None) -> AIResponse:
        payload = {"model": self._model, "messages": [dict(m) for m in messages], "max_tokens": max_tokens,
                   "json_format": json_format or json_schema is not None}
        if json_schema is not None:
            payload["json_schema"] = json_schema
        try:
            data = await post_json(f"{self._base_url}/dialog/", payload)
        except HTTPError as exc:
            raise Exception(f"Failed to get response. Got status code {exc.status} from GPU Service with message "
                            f"{exc.body}") from exc
        self._record_attempts(1)
        return AIResponse(**data["response"])
