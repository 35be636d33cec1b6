"""Ollama embeddings, one request per text (reference ai/embedders/ollama.py:8-22)."""
from __future__ import annotations

from typing import List

from assistant.ai.providers._http import post_json
from assistant.ai.providers.base import AIEmbedder


class OllamaEmbedder(AIEmbedder):
    def __init__(self, host: str, model: str):
        self._host, self._model = host.rstrip("/"), model

    async def embeddings(self, input: List[str]) -> List[List[float]]:
        out = []
        for text in input:
            data = await post_json(f"{self._host}/api/embeddings", {"model": self._model, "prompt": text})
            out.append(data["embedding"])
        return out
