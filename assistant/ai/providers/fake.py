"""Deterministic offline providers for tests, demos and benchmarks (model names ``test`` / ``fake:*``).

The reference tests mock the AI at the bot boundary and use ``DEFAULT_AI_MODEL='test'``
(tests/settings.py:132) without a matching provider; here ``test`` resolves to these classes:
  * FakeAIProvider -- scripted responses (``FakeAIProvider.script([...])``), else an echo of the last
    user message; in JSON mode it answers with the first example schema found in the prompt, so the
    JSON-validated pipeline steps (classify, known-question choice, ...) run end to end offline.
  * FakeEmbedder   -- hashed bag-of-words vectors: identical texts embed identically, texts sharing
    words are close under cosine, no model needed.
"""
from __future__ import annotations

import hashlib
import json
import re
from collections import deque
from typing import List

import numpy as np

from assistant.ai.domain import AIResponse, Message
from assistant.ai.providers.base import AIEmbedder, AIProvider

_JSON_BLOCK = re.compile(r"```json\s*(.*?)```", re.S)
_COMMENT = re.compile(r"//[^\n]*")


def parse_example_json(text: str):
    """Parse a prompt's example schema: strips // comments, '...' lines and trailing commas."""
    body = _COMMENT.sub("", text)
    body = "\n".join(line for line in body.splitlines() if line.strip() not in ("...", "..."))
    body = re.sub(r",(\s*[\]}])", r"\1", body)
    return json.loads(body)


class FakeAIProvider(AIProvider):
    _script: deque = deque()
    requests: list = []

    def __init__(self, model: str = "test"):
        self._model = model

    @classmethod
    def script(cls, responses: list) -> None:
        cls._script.extend(responses)

    @classmethod
    def reset(cls) -> None:
        cls._script.clear()
        cls.requests.clear()

    @property
    def context_size(self) -> int:
        return 8000

    def calculate_tokens(self, text: str) -> int:
        return len(text.split()) // 2

    async def get_response(self, messages: List[Message], max_tokens: int = 1024,
                           json_format: bool = False, json_schema: dict | None = None) -> AIResponse:
        FakeAIProvider.requests.append({"messages": list(messages), "max_tokens": max_tokens,
                                        "json_format": json_format, "json_schema": json_schema})
        json_format = json_format or json_schema is not None
        if self._script:
            r = self._script.popleft()
            result = r(messages) if callable(r) else r
        elif json_format:
            result = {}
            for m in reversed(messages):
                blocks = _JSON_BLOCK.findall(m.get("content") or "")
                if blocks:
                    try:
                        result = parse_example_json(blocks[0])
                    except json.JSONDecodeError:
                        pass
                    break
        else:
            last = next((m["content"] for m in reversed(messages) if m["role"] == "user"), "")
            result = f"Test AI response: {last}"[: max(16, max_tokens * 4)]
        if isinstance(result, AIResponse):
            return result
        n_in = sum(len((m.get("content") or "").split()) for m in messages)
        n_out = len(json.dumps(result).split()) if isinstance(result, dict) else len(str(result).split())
        self._record_attempts(1)
        return AIResponse(result=result, usage={"model": self._model, "prompt_tokens": n_in,
                                                "completion_tokens": n_out})


class FakeEmbedder(AIEmbedder):
    def __init__(self, model: str = "test", dim: int = 768):
        self._model = model
        self.dim = dim

    def _word_vec(self, w: str) -> np.ndarray:
        seed = int.from_bytes(hashlib.blake2b(w.encode(), digest_size=8).digest(), "little")
        return np.random.default_rng(seed).standard_normal(self.dim)

    def embed_one(self, text: str) -> list:
        words = re.findall(r"\w+", (text or "").lower())
        v = np.zeros(self.dim)
        for w in words:
            v += self._word_vec(w)
        n = np.linalg.norm(v)
        if n == 0:
            v = self._word_vec("<empty>")
            n = np.linalg.norm(v)
        return (v / n).astype(np.float32).tolist()

    async def embeddings(self, input: List[str]) -> List[List[float]]:
        return [self.embed_one(t) for t in input]
