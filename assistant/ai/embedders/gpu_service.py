"""Client of the gpu_service ``POST /embeddings/`` endpoint (reference ai/embedders/gpu_service.py:8-28)."""
from __future__ import annotations

from typing import List

from assistant.ai.providers._http import HTTPError, post_json
from assistant.ai.providers.base import AIEmbedder


class GPUServiceEmbedder(AIEmbedder):
    def __init__(self, base_url: str, model: str):
        self._base_url = base_url.rstrip("/")
        self._model = model

    async def embeddings(self, input: List[str]) -> List[List[float]]:
        try:
            data = await post_json(f"{self._base_url}/embeddings/", {"model": self._model, "texts": list(input)})
        except HTTPError as exc:
            raise Exception(f"Failed to get embeddings. Got status code {exc.status} from GPU Service with message "
                            f"{exc.body}") from exc
        return data["embeddings"]
