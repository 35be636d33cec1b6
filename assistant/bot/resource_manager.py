"""Per-bot prompts, messages and phrases with language fallback (reference bot/resource_manager.py).
Fixes the reference's phrase fallback, which returned the raw JSON file text instead of the phrase."""
from __future__ import annotations

import json
import logging
import os

from assistant.bot.domain import NoMessageFound, NoResourceFound
from assistant.conf import settings

logger = logging.getLogger(__name__)


class ResourceManager:
    def __init__(self, codename: str, language: str, default_language: str = None):
        self.codename = codename
        self.language = language
        self.default_language = default_language or settings.get("BOT_DEFAULT_LANGUAGE", "ru")

    def get_resource(self, path: str) -> str:
        file_path = os.path.join(str(settings.RESOURCES_DIR), self.codename, path)
        try:
            with open(file_path, encoding="utf-8") as f:
                return f.read()
        except FileNotFoundError:
            raise NoResourceFound(file_path)

    def get_prompt(self, path: str) -> str:
        return self.get_resource(f"prompts/{path}")

    def get_message(self, path: str) -> str:
        for lang in (self.language, self.default_language):
            try:
                return self.get_resource(f"messages/{lang}/{path}")
            except NoResourceFound as e:
                logger.debug("message %s missing for %s: %s", path, lang, e)
        raise NoMessageFound(path)

    def _phrases(self, lang: str) -> dict:
        try:
            return json.loads(self.get_resource(f"phrases/{lang}.json"))
        except NoResourceFound:
            return {}
        except json.JSONDecodeError:
            logger.exception("invalid phrases file for %s", lang)
            return {}

    def get_phrase(self, phrase: str) -> str:
        for lang in (self.language, self.default_language):
            value = self._phrases(lang).get(phrase)
            if value is not None:
                return value
        return phrase
