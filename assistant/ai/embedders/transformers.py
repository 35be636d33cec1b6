"""In-process sentence embeddings on the MI355X engine (replaces the reference's per-text HF loop,
ai/embedders/transformers.py:8-29).  Concurrent callers are batched into packed variable-length
encoder batches by ``EmbedWorker``; pooling is the reference's mean over all tokens, truncation to
the model's 512 positions is applied (the reference crashed on longer texts)."""
from __future__ import annotations

from typing import List

from assistant.ai.providers.base import AIEmbedder


class TransformersEmbedder(AIEmbedder):
    def __init__(self, model_name: str, local_files_only: bool = True, **engine_kwargs):
        from django_assistant_bot_amd.engine.serving import get_embed_worker

        self._model = model_name
        self._worker = get_embed_worker(model_name, **engine_kwargs)

    @property
    def dim(self) -> int:
        return self._worker.engine.dim

    async def embeddings(self, input: List[str]) -> List[List[float]]:
        return await self._worker.embeddings(list(input))
