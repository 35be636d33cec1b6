"""Prefix-routed provider / embedder factories, tagged-text extraction and cost accounting
(reference ai/services/ai_service.py:14-122).

Providers:  ``groq:<m>`` Groq | ``gpu_service:<m>`` gpu_service HTTP | ``engine:<m>`` in-process MI355X
engine | ``llama*`` / ``ollama:<m>`` Ollama | ``test`` / ``fake:<m>`` offline fake | else OpenAI.
Embedders:  ``text-embedding-3*`` OpenAI | ``gpu_service:<m>`` | ``engine:<m>`` | ``test`` / ``fake:<m>`` |
else Ollama (default model ``nomic-embed-text``).
Engine-backed objects are cached per model (one engine per process); HTTP clients are cheap.
"""
from __future__ import annotations

import logging
import re
from decimal import Decimal
from typing import Dict

from assistant.ai.providers.base import AIEmbedder, AIProvider
from assistant.conf import settings

logger = logging.getLogger(__name__)


def get_ai_provider(model: str) -> AIProvider:
    logger.debug("AI provider for model %s", model)
    if model == "test" or model.startswith("fake:"):
        from assistant.ai.providers.fake import FakeAIProvider

        return FakeAIProvider(model)
    if model.startswith("groq:"):
        from assistant.ai.providers.groq import GroqAIProvider

        return GroqAIProvider(model=model[len("groq:"):], api_key=settings.GROQ_API_KEY,
                              base_url=settings.get("GROQ_BASE_URL", "https://api.groq.com/openai/v1"))
    if model.startswith("gpu_service:"):
        from assistant.ai.providers.gpu_service import GPUServiceProvider

        return GPUServiceProvider(base_url=settings.GPU_SERVICE_ENDPOINT, model=model[len("gpu_service:"):])
    if model.startswith("engine:"):
        from assistant.ai.providers.transformers import TransformersProvider

        return TransformersProvider(model[len("engine:"):])
    if model.startswith("llama"):
        from assistant.ai.providers.ollama import OllamaAIProvider

        return OllamaAIProvider(model=model, host=settings.OLLAMA_ENDPOINT)  # prefix kept (reference behaviour)
    if model.startswith("ollama:"):
        from assistant.ai.providers.ollama import OllamaAIProvider

        return OllamaAIProvider(model=model[len("ollama:"):], host=settings.OLLAMA_ENDPOINT)
    from assistant.ai.providers.openai import ChatGPTAIProvider

    return ChatGPTAIProvider(model=model, api_key=settings.OPENAI_API_KEY,
                             base_url=settings.get("OPENAI_BASE_URL", "https://api.openai.com/v1"))


def get_ai_embdedder(model: str = None) -> AIEmbedder:
    """(sic) the reference's public name; ``get_ai_embedder`` is an alias."""
    model = model or "nomic-embed-text"
    if model == "test" or model.startswith("fake:"):
        from assistant.ai.providers.fake import FakeEmbedder

        return FakeEmbedder(model)
    if model.startswith("text-embedding-3"):
        from assistant.ai.embedders.openai import ChatGPTEmbedder

        return ChatGPTEmbedder(model=model, api_key=settings.OPENAI_API_KEY,
                               base_url=settings.get("OPENAI_BASE_URL", "https://api.openai.com/v1"))
    if model.startswith("gpu_service:"):
        from assistant.ai.embedders.gpu_service import GPUServiceEmbedder

        return GPUServiceEmbedder(base_url=settings.GPU_SERVICE_ENDPOINT, model=model[len("gpu_service:"):])
    if model.startswith("engine:"):
        from assistant.ai.embedders.transformers import TransformersEmbedder

        return TransformersEmbedder(model[len("engine:"):])
    from assistant.ai.embedders.ollama import OllamaEmbedder

    return OllamaEmbedder(model=model, host=settings.OLLAMA_ENDPOINT)


get_ai_embedder = get_ai_embdedder

_TAG = re.compile(r"#(\w+)\s?(.*?)(?=\s#|$)", re.S)


def extract_tagged_text(text: str) -> Dict[str, str]:
    """'#tag text #other more' -> {'tag': 'text', 'other': 'more'} (tags lower-cased)."""
    return {tag.lower(): body.strip() for tag, body in _TAG.findall(text or "")}


_DALLE = {("1024x1024", "standard"): Decimal("0.04"), ("1024x1792", "standard"): Decimal("0.08"),
          ("1792x1024", "standard"): Decimal("0.08"), ("1024x1024", "hd"): Decimal("0.08"),
          ("1024x1792", "hd"): Decimal("0.12"), ("1792x1024", "hd"): Decimal("0.12")}
# USD per 1K tokens (prompt, completion)
_PER_1K = (("gpt-3.5-turbo", Decimal("0.001"), Decimal("0.002")), ("gpt-4-", Decimal("0.01"), Decimal("0.03")))


def calculate_ai_cost(usage: Dict) -> Decimal:
    model = (usage or {}).get("model") or ""
    if model == "dall-e-3":
        size = usage["size"].replace("×", "x")
        return _DALLE[(size, usage["quality"])] * usage["n"]
    for prefix, p_in, p_out in _PER_1K:
        if model.startswith(prefix):
            return (p_in * usage.get("prompt_tokens", 0) + p_out * usage.get("completion_tokens", 0)) / 1000
    if model.startswith("llama") or model == "test" or model.startswith(("fake:", "engine:")):
        return Decimal(0)
    logger.warning("Unknown model for cost: %s", model)
    return Decimal(0)
