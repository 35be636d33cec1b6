"""Interactive console chat with a bot, stored in the database like any platform
(reference bot/management/commands/chat.py).  ``--memory`` runs without touching the database.  Like the
reference, the chat restarts when a source file changes (``--noreload`` disables it)."""
import asyncio
import json
import logging
import os
import uuid
from datetime import timedelta

from django.core.management import BaseCommand
from django.db.models import Max

from assistant.bot.domain import User
from assistant.bot.platforms.console import ConsolePlatform
from assistant.bot.session import BotSession
from assistant.bot.utils import get_bot_class
from assistant.utils.sync import sync_to_async

HISTORY_FILE_NAME = ".chat_history.jsonl"


def load_readline_history(path: str):
    try:
        import readline
    except ImportError:
        return
    if not os.path.exists(path):
        return
    with open(path, encoding="utf-8") as f:
        for line in f:
            try:
                rec = json.loads(line)
            except json.JSONDecodeError:
                continue
            if rec.get("role") == "user":
                readline.add_history(rec.get("text", ""))


class Command(BaseCommand):
    help = "Interactive chat with a bot through the console (debugging)"

    def add_arguments(self, parser):
        parser.add_argument("bot_codename")
        parser.add_argument("--memory", action="store_true", help="in-memory dialog (no database writes)")
        parser.add_argument("--history", default=HISTORY_FILE_NAME)
        parser.add_argument("--noreload", action="store_true", help="do not restart on code changes")

    def handle(self, *args, **opts):
        if opts["noreload"]:
            return self._chat(opts)
        from assistant.utils.autoreload import run_with_reloader

        run_with_reloader(self._chat, opts)

    def _chat(self, opts):
        logging.getLogger().setLevel(logging.WARNING)
        codename = opts["bot_codename"]
        platform = ConsolePlatform(opts["history"])
        bot_cls = get_bot_class(codename)
        loop = asyncio.new_event_loop()
        asyncio.set_event_loop(loop)
        if opts["memory"]:
            session = BotSession.in_memory(bot_cls, platform, codename=codename)
        else:
            session = loop.run_until_complete(self._db_session(codename, bot_cls, platform))
        load_readline_history(opts["history"])
        self.stdout.write(f"Interactive chat with bot '{codename}' (exit / quit / Ctrl-D to leave)")
        while True:
            try:
                text = input("\nYou: ")
            except (EOFError, KeyboardInterrupt):
                break
            if text.strip().lower() in ("exit", "quit"):
                break
            platform.record({"role": "user", "text": text})
            loop.run_until_complete(session.send(text))
        loop.close()

    async def _db_session(self, codename, bot_cls, platform):
        from assistant.bot.management.commands.utils import get_instance
        from assistant.bot.models import Message
        from assistant.bot.services.dialog_service import get_dialog
        from assistant.bot.services.instance_service import InstanceLockAsync
        from assistant.bot.store import DjangoBotStore

        chat_id = str(uuid.uuid4())
        user = User(id=chat_id, username="tester", first_name="Test", last_name="User", language_code="ru")
        instance = await sync_to_async(get_instance)(codename, "console", chat_id, user)
        dialog = await sync_to_async(get_dialog)(instance, timedelta(days=1))
        session = BotSession(bot_cls, platform, DjangoBotStore(), dialog, user=user, chat_id=chat_id,
                             lock_factory=InstanceLockAsync)
        session.message_id = await sync_to_async(
            lambda: Message.objects.filter(dialog=dialog).aggregate(Max("id"))["id__max"] or 0)()
        return session
