"""Drive a bot outside the webhook: console chat, self-play testing, tests.

``BotSession`` owns one (bot, platform, store, dialog) and feeds text turns through the same
``answer_update`` path as the Celery task, numbering message ids itself.  With ``MemoryBotStore`` it
needs no database (``python -m assistant.bot.session`` starts an in-memory console chat).
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import uuid
from typing import Optional, Type

from assistant.bot.domain import BotPlatform, SingleAnswer, Update, User
from assistant.bot.resource_manager import ResourceManager
from assistant.bot.services.answer_service import answer_update
from assistant.bot.store import BotRecord, BotUserRecord, InstanceRecord, MemoryBotStore

logger = logging.getLogger(__name__)


class BotSession:
    def __init__(self, bot_cls: Type, platform: BotPlatform, store, dialog, user: Optional[User] = None,
                 chat_id: Optional[str] = None, lock_factory=None, error_language: str = "ru"):
        self.bot_cls = bot_cls
        self.platform = platform
        self.store = store
        self.dialog = dialog
        self.chat_id = chat_id or str(uuid.uuid4())
        self.user = user or User(id=self.chat_id, username="tester", first_name="Test", last_name="User",
                                 language_code=error_language)
        self.lock_factory = lock_factory
        self.error_language = error_language
        self.message_id = 0
        self.turns = 0

    @classmethod
    def in_memory(cls, bot_cls: Type, platform: BotPlatform, codename: str = "default", system_text: str = None,
                  start_text: str = None, help_text: str = None, user_id: str = "console", language: str = "ru"):
        store = MemoryBotStore()
        bot = BotRecord(codename=codename, system_text=system_text, start_text=start_text, help_text=help_text)
        instance = InstanceRecord(bot=bot, user=BotUserRecord(user_id=user_id, platform=platform.codename,
                                                              username="@tester", language=language))
        return cls(bot_cls, platform, store, store.open_dialog(instance), chat_id=user_id,
                   error_language=language)

    def _error_answer(self, phrase: str) -> SingleAnswer:
        rm = ResourceManager(codename=self.dialog.instance.bot.codename, language=self.error_language)
        return SingleAnswer(rm.get_phrase(phrase), no_store=True)

    async def send(self, text: str):
        """One user turn; returns the bot's answer (already posted to the platform) or None."""
        self.message_id += 1
        self.turns += 1
        update = Update(chat_id=self.chat_id, message_id=self.message_id, text=text, user=self.user)
        await self.store.add_user_message(self.dialog, update.message_id, update.text)
        bot = self.bot_cls(dialog=self.dialog, platform=self.platform, store=self.store)
        lock = self.lock_factory(self.dialog.instance) if self.lock_factory else None
        try:
            return await answer_update(bot, self.platform, update, lock=lock, instance_is_new=self.turns == 1)
        except Exception:
            logger.exception("Error while handling update")
            answer = self._error_answer("An error occurred while processing your message.")
            await self.platform.post_answer(self.chat_id, answer)
            return answer


def _main():  # pragma: no cover - interactive
    from assistant.bot.platforms.console import ConsolePlatform
    from assistant.bot.utils import get_bot_class
    from assistant.conf import configure

    p = argparse.ArgumentParser(description="In-memory console chat with a bot (no database)")
    p.add_argument("--bot", default="default")
    p.add_argument("--model", default=None, help="AI model id (e.g. 'test', 'engine:llama-3-8b', 'groq:...')")
    p.add_argument("--system", default=None)
    p.add_argument("--history", default=".chat_history.jsonl")
    args = p.parse_args()
    if args.model:
        configure(DEFAULT_AI_MODEL=args.model)
    session = BotSession.in_memory(get_bot_class(args.bot), ConsolePlatform(args.history), codename=args.bot,
                                   system_text=args.system)
    loop = asyncio.new_event_loop()
    print(f"Interactive chat with bot '{args.bot}' (exit / quit / Ctrl-D to leave)")
    while True:
        try:
            text = input("\nYou: ")
        except (EOFError, KeyboardInterrupt):
            break
        if text.strip().lower() in ("exit", "quit"):
            break
        session.platform.record({"role": "user", "text": text})
        loop.run_until_complete(session.send(text))
    loop.close()


if __name__ == "__main__":  # pragma: no cover
    _main()
