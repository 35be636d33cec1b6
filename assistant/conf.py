"""Settings access that works with and without Django.

Inside a Django project ``settings.X`` reads ``django.conf.settings.X``.  Without a configured Django
(engine-only deployments, unit tests) it falls back to values set with :func:`configure`, then to
environment variables, then to the defaults below (reference Appendix B keys).
"""
from __future__ import annotations

import os
from typing import Any

DEFAULTS: dict[str, Any] = {
    "DEFAULT_AI_MODEL": "test",
    "EMBEDDING_AI_MODEL": "test",
    "DOCUMENT_MAX_LENGTH": 1000,
    "BOT_DEFAULT_LANGUAGE": "ru",
    "BOTS": {},
    "DOCUMENT_PROCESSOR_CLASSES": {},
    "GPU_SERVICE_ENDPOINT": "http://127.0.0.1:11435",
    "OLLAMA_ENDPOINT": "http://127.0.0.1:11434",
    "OPENAI_API_KEY": "",
    "OPENAI_BASE_URL": "https://api.openai.com/v1",
    "GROQ_API_KEY": "",
    "GROQ_BASE_URL": "https://api.groq.com/openai/v1",
    "TELEGRAM_API_URL": "https://api.telegram.org",
    "TELEGRAM_BASE_CALLBACK_URL": "",
    "RESOURCES_DIR": "resources",
    "DEBUG": False,
    # engine settings
    "GPU_SERVICE_DEVICES": None,
    # gpu_service node mode (gpu_service/node_main.py): ranks holding an encoder replica / an index
    # shard (0 = every GPU of the node) and the generator's tensor-parallel degree
    "EMBED_DP": 0,
    "GEN_TP": 1,
    "KV_BLOCK_SIZE": 64,
    "MAX_BATCH_TOKENS": 65536,
    "INDEX_SHARDS": 0,
    "INDEX_DTYPE": "bfloat16",
    "ENGINE_RANDOM_WEIGHTS": True,
    # engine: apply a checkpoint's chat template (tokenizer_config.json) instead of the reference's
    # "role: content" prompt lines
    "ENGINE_CHAT_TEMPLATE": False,
}

_overrides: dict[str, Any] = {}


def _django_settings():
    try:
        from django.conf import settings as dj

        if dj.configured:
            return dj
    except Exception:
        return None
    return None


class _Settings:
    def __getattr__(self, name: str) -> Any:
        if name.startswith("__"):
            raise AttributeError(name)
        dj = _django_settings()
        if dj is not None and hasattr(dj, name):
            return getattr(dj, name)
        if name in _overrides:
            return _overrides[name]
        if name in os.environ:
            return os.environ[name]
        if name in DEFAULTS:
            return DEFAULTS[name]
        raise AttributeError(f"setting {name} is not defined")

    def get(self, name: str, default: Any = None) -> Any:
        try:
            return getattr(self, name)
        except AttributeError:
            return default


settings = _Settings()


def configure(**values: Any) -> None:
    _overrides.update(values)


def reset(*names: str) -> None:
    for n in names or list(_overrides):
        _overrides.pop(n, None)
