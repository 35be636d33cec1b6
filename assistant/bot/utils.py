"""Bot helpers: platform / bot-class resolution (reference bot/utils.py:16-70)."""
from __future__ import annotations

import importlib
import logging
from functools import lru_cache

from assistant.conf import settings
from assistant.utils.repeat_until import MaxAttemptsExceededError  # noqa: F401  (re-export, API compat)

logger = logging.getLogger(__name__)

DEFAULT_BOT_CLASS = "assistant.bot.assistant_bot.AssistantBot"


def truncate_text(text: str, max_tokens: int = 1024) -> str:
    words = (text or "").split()
    if len(words) > max_tokens:
        return " ".join(words[:max_tokens]) + "..."
    return text


def get_bot_platform(bot_codename: str, platform_codename: str):
    """Telegram platform with the token from ``settings.BOTS`` (preferred) or the Bot row.
    Non-telegram platform codenames (e.g. the REST API's 'default_platform') return None."""
    from django.http import Http404

    from assistant.bot.models import Bot as BotModel
    from assistant.bot.platforms.telegram.platform import TelegramBotPlatform

    cfg = settings.get("BOTS", {}) or {}
    token = (cfg.get(bot_codename) or {}).get("telegram_token")
    if token:
        return TelegramBotPlatform(token)
    if platform_codename != "telegram":
        return None
    token = BotModel.objects.filter(codename=bot_codename).values_list("telegram_token", flat=True).first()
    if not token:
        raise Http404("Bot not found")
    return TelegramBotPlatform(token)


@lru_cache
def get_bot_class(bot_codename: str):
    cfg = settings.get("BOTS", {}) or {}
    path = (cfg.get(bot_codename) or {}).get("class")
    if not path:
        path = (settings.get("BOT_CLASSES", {}) or {}).get(bot_codename) or settings.get("DEFAULT_BOT_CLASS",
                                                                                           DEFAULT_BOT_CLASS)
    logger.info("bot class %s for %s", path, bot_codename)
    return import_string(path)


def import_string(path: str):
    """``pkg.module.Name`` -> object (django.utils.module_loading.import_string without Django)."""
    module_path, _, name = path.rpartition(".")
    return getattr(importlib.import_module(module_path), name)
