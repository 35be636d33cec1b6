"""Django / Celery / DRF modules cannot be imported here (those packages are not installed), so
every application module is at least byte-compiled, and the Django-free modules are imported."""
import importlib
import pathlib
import py_compile

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
APP_FILES = sorted(p for d in ("assistant", "gpu_service", "example") for p in (ROOT / d).rglob("*.py"))


@pytest.mark.parametrize("path", APP_FILES, ids=lambda p: str(p.relative_to(ROOT)))
def test_compiles(path):
    py_compile.compile(str(path), doraise=True)


DJANGO_FREE = [
    "assistant.conf", "assistant.utils.sync", "assistant.utils.autoreload", "assistant.utils.tasks", "assistant.utils.language",
    "assistant.utils.fuzzy", "assistant.utils.repeat_until", "assistant.ai.services.ai_service",
    "assistant.bot.domain", "assistant.bot.assistant_bot", "assistant.bot.store", "assistant.bot.session",
    "assistant.bot.selfplay", "assistant.bot.tasks", "assistant.bot.services.answer_service",
    "assistant.bot.platforms.telegram.platform", "assistant.bot.platforms.console", "assistant.bot.platforms.api",
    "assistant.bot.chat_completion", "assistant.rag.knowledge", "assistant.rag.aggregation",
    "assistant.assistant.queue", "assistant.processing.utils", "assistant.processing.repository",
    "assistant.processing.wiki", "assistant.processing.documents.processor", "assistant.broadcasting.core",
    "assistant.loading.csv_loader", "assistant.loading.csv", "gpu_service.main", "gpu_service.models",
]


@pytest.mark.parametrize("mod", DJANGO_FREE)
def test_imports_without_django(mod):
    importlib.import_module(mod)
