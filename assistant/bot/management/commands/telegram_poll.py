"""Run a bot in Telegram long-polling mode (reference bot/management/commands/telegram_poll.py).

Uses ``getUpdates`` of the raw Bot API client (no python-telegram-bot).  Each update is stored like a
webhook update and answered through ``answer_task`` -- inline with ``--sync``, else via Celery.
``--dev`` restarts the poller when a source file changes (``assistant.utils.autoreload``)."""
import asyncio
import logging
from datetime import timedelta

from django.core.management import BaseCommand

from assistant.bot.domain import UnknownUpdate
from assistant.bot.management.commands.utils import get_instance
from assistant.bot.services.dialog_service import create_user_message, get_dialog
from assistant.bot.tasks import _answer_task, answer_task
from assistant.bot.utils import get_bot_platform
from assistant.utils.sync import sync_to_async

logger = logging.getLogger(__name__)


class Command(BaseCommand):
    help = "Run a bot in Telegram polling mode"

    def add_arguments(self, parser):
        parser.add_argument("bot_codename")
        parser.add_argument("--sync", action="store_true", help="answer inline instead of through Celery")
        parser.add_argument("--timeout", type=int, default=30, help="long-poll timeout (s)")
        parser.add_argument("--dev", action="store_true", help="development mode: auto-reload on code changes")

    def handle(self, *args, **opts):
        if opts["dev"]:
            from assistant.utils.autoreload import run_with_reloader

            logger.info("development mode: auto-reload enabled")
            run_with_reloader(self._run, opts)
        else:
            self._run(opts)

    def _run(self, opts):
        try:
            asyncio.run(self._poll(opts["bot_codename"], opts["sync"], opts["timeout"]))
        except KeyboardInterrupt:
            self.stdout.write("\nBot stopped")

    async def _poll(self, codename: str, sync_mode: bool, timeout: int):
        platform = await sync_to_async(get_bot_platform)(codename, "telegram")
        await platform.api.call("deleteWebhook")  # getUpdates is refused while a webhook is set
        self.stdout.write(f"Bot '{codename}' polling Telegram ({'sync' if sync_mode else 'celery'} mode)")
        offset = None
        while True:
            try:
                updates = await platform.get_updates(offset=offset, timeout=timeout)
            except Exception:
                logger.exception("getUpdates failed; retrying in 5 s")
                await asyncio.sleep(5)
                continue
            for raw in updates or []:
                offset = raw["update_id"] + 1
                try:
                    update = await platform.convert_telegram_update(raw)
                except UnknownUpdate:
                    continue
                except Exception:
                    logger.exception("cannot convert update %s", raw.get("update_id"))
                    continue
                try:
                    await self._process(codename, platform, update, sync_mode)
                except Exception:
                    logger.exception("error processing update for chat %s", update.chat_id)

    async def _process(self, codename, platform, update, sync_mode):
        instance = await sync_to_async(get_instance)(codename, "telegram", update.chat_id, update.user)
        dialog = await sync_to_async(get_dialog)(instance, timedelta(days=1))
        await sync_to_async(create_user_message)(dialog, update.message_id, update.text, update.photo,
                                                 update.phone_number)
        await platform.action_typing(update.chat_id)
        if sync_mode:
            await _answer_task(codename, str(dialog.id), "telegram", update.to_dict())
        else:
            answer_task.delay(codename, str(dialog.id), "telegram", update.to_dict())
