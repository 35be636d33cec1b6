"""Platform webhooks (reference bot/views.py:26-120).

A webhook request is parsed into an ``Update``, the bot user / instance / dialog are resolved (the
dialog rotates after a day of silence), the user message is stored, and the answer is produced
asynchronously by ``answer_task`` on the query queue.  Telegram always gets 200 so it does not retry.
"""
import logging
from abc import ABC, abstractmethod
from datetime import timedelta

from rest_framework.permissions import AllowAny
from rest_framework.response import Response
from rest_framework.views import APIView

from assistant.bot.adrf import AsyncMixin
from assistant.bot.domain import UnknownUpdate, Update, User
from assistant.bot.models import Bot, BotUser, Instance
from assistant.bot.services.dialog_service import create_user_message, get_dialog
from assistant.bot.tasks import answer_task
from assistant.bot.utils import get_bot_platform
from assistant.conf import settings
from assistant.utils.sync import sync_to_async

logger = logging.getLogger(__name__)

DIALOG_TTL = timedelta(days=1)


def display_username(user: User):
    if user.username:
        return "@" + user.username
    name = " ".join(p for p in (user.first_name, user.last_name) if p)
    return name or None


def get_or_create_instance(codename: str, platform_codename: str, update: Update):
    bot = Bot.objects.filter(codename=codename).first()
    if bot is None:
        if codename not in (settings.get("BOTS") or {}):
            raise Bot.DoesNotExist(codename)
        bot = Bot.objects.create(codename=codename)
    user = update.user
    language = user.language_code if user else None
    username = display_username(user) if user else None
    bot_user, _ = BotUser.objects.get_or_create(user_id=update.chat_id, platform=platform_codename,
                                                defaults={"username": username, "language": language})
    changed = [f for f, v in (("language", language), ("username", username)) if getattr(bot_user, f) != v]
    for f in changed:
        setattr(bot_user, f, language if f == "language" else username)
    if changed:
        bot_user.save(update_fields=changed)
    instance, created = Instance.objects.get_or_create(user_id=bot_user.id, bot_id=bot.id)
    return Instance.objects.select_related("bot", "user").get(id=instance.id), created


class BaseAssistantBotView(AsyncMixin, APIView, ABC):
    @abstractmethod
    def get_bot_codename(self, request) -> str: ...

    @abstractmethod
    def get_platform_codename(self, request) -> str: ...

    async def post(self, request, **kwargs):
        bot_codename = self.get_bot_codename(request)
        platform_codename = self.get_platform_codename(request)
        platform = await sync_to_async(get_bot_platform)(bot_codename, platform_codename)
        try:
            update = await platform.get_update(request)
        except UnknownUpdate:
            logger.info("Ignoring unknown update")
            return Response(status=200)
        try:
            dialog = await self._get_dialog(bot_codename, platform_codename, update)
        except Exception:
            logger.exception("Cannot resolve dialog")
            return Response(status=200)
        answer_task.delay(bot_codename, str(dialog.id), platform_codename, update.to_dict())
        return Response(status=200)

    async def _get_dialog(self, bot_codename, platform_codename, update):
        instance, _ = await sync_to_async(get_or_create_instance)(bot_codename, platform_codename, update)
        dialog = await sync_to_async(get_dialog)(instance, DIALOG_TTL)
        await sync_to_async(create_user_message)(dialog, update.message_id, update.text, update.photo,
                                                 update.phone_number)
        return dialog


class TelegramAssistantBotView(BaseAssistantBotView):
    permission_classes = [AllowAny]

    def get_bot_codename(self, request) -> str:
        return self.kwargs.get("codename", "")

    def get_platform_codename(self, request) -> str:
        return "telegram"
