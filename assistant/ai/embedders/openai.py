"""OpenAI embeddings, one batched request (reference ai/embedders/openai.py:8-25)."""
from __future__ import annotations

from typing import List

from assistant.ai.providers._http import post_json
from assistant.ai.providers.base import AIEmbedder


class ChatGPTEmbedder(AIEmbedder):
    def __init__(self, model: str, api_key: str, base_url: str = "https://api.openai.com/v1"):
        self._model, self._api_key, self._base_url = model, api_key, base_url.rstrip("/")

    async def embeddings(self, input: List[str]) -> List[List[float]]:
        data = await post_json(f"{self._base_url}/embeddings", {"model": self._model, "input": list(input)},
                               headers={"Authorization": f"Bearer {self._api_key}"})
        return [d["embedding"] for d in sorted(data["data"], key=lambda d: d.get("index", 0))]
