"""Provider / embedder interfaces and the AI call debugger (reference ai/providers/base.py:8-70)."""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import List, Optional

from assistant.ai.domain import AIResponse, Message
from assistant.utils.debug import TimeDebugger


def accepts_json_schema(fn) -> bool:
    """Whether a ``get_response`` takes the ``json_schema`` keyword (custom providers written for the
    reference's ``(messages, max_tokens, json_format)`` signature do not)."""
    import inspect

    try:
        params = inspect.signature(fn).parameters
    except (TypeError, ValueError):
        return False
    return "json_schema" in params or any(p.kind == p.VAR_KEYWORD for p in params.values())


class AIProvider(ABC):
    #: per-call attempt counts, recorded when a debugger asks for them (None = not recording)
    calls_attempts: Optional[List[int]] = None

    @property
    @abstractmethod
    def context_size(self) -> int:
        """Context window of the model in tokens."""

    @abstractmethod
    def calculate_tokens(self, text: str) -> int:
        """Token count of ``text`` for this model."""

    @abstractmethod
    async def get_response(self, messages: List[Message], max_tokens: int = 1024,
                           json_format: bool = False, json_schema: dict | None = None) -> AIResponse:
        """Chat completion for ``messages``.  ``json_schema`` (an extension of the reference API):
        a JSON Schema the answer must follow; providers that can enforce it do (the MI355X engine
        by constrained decoding, OpenAI / Ollama by their structured-output options), the others
        treat it as ``json_format``."""

    def _record_attempts(self, n: int) -> None:
        if self.calls_attempts is not None:
            self.calls_attempts.append(n)


class AIEmbedder(ABC):
    @abstractmethod
    async def embeddings(self, input: List[str]) -> List[List[float]]:
        """One vector per input text."""


class AIDebugger(TimeDebugger):
    """Times an AI call and records the attempts the provider needed and the model used."""

    def __init__(self, ai: AIProvider, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.ai = ai
        self._attempts = None

    def __enter__(self):
        self.ai.calls_attempts = []
        return super().__enter__()

    @property
    def call_attempts(self):
        if self._attempts is not None:
            return self._attempts
        ca = getattr(self.ai, "calls_attempts", None)
        return sum(ca) if ca is not None else None

    def __exit__(self, exc_type, exc, tb):
        super().__exit__(exc_type, exc, tb)
        self._attempts = self.call_attempts
        self.info["attempts"] = self._attempts
        self.info["model"] = getattr(self.ai, "_model", None)
        return False
